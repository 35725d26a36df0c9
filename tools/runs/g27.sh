set -o pipefail
out=gpurun_out/g27
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest.log python -u -m pytest tests/test_gpu_range_coder.py -m gpu -x -v --timeout 200 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
tools/gpu_step.sh 300 $out/rc.log python -u tools/rc_bench.py || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/rc_trace -o run --output-format csv -- python3 tools/rc_bench.py --reps 2 > $out/rc_rocprof.log 2>&1 || exit 1
