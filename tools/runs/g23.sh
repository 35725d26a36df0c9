set -o pipefail
out=gpurun_out/g23
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest.log python -u -m pytest tests/test_gpu_fragments.py -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
tools/gpu_step.sh 200 $out/frag.log python -u tools/frag_bench.py || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/frag_trace -o run --output-format csv -- python3 tools/frag_bench.py --reps 10 > $out/frag_rocprof.log 2>&1 || exit 1
