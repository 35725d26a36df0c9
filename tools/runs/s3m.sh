set -o pipefail
# round 2 (session 4): gather lists via a length-binned segment pass + join -- parity, then cfg5 throughput
out=gpurun_out/s3m
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gather" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/gather.json python -u tools/gather_bench.py || exit 1
tools/gpu_step.sh 300 $out/gather_l4.json python -u tools/gather_bench.py --lanes 4 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/gather_bench.py > $out/gather_under_rocprof.json 2>&1 || exit 1
