set -o pipefail
# round 2 (session 4): verify lists via the vring checksum pass + a fix-up launch -- parity, throughput
out=gpurun_out/s3q
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "verify" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
tools/gpu_step.sh 200 $out/verify_l5.json python -u tools/verify_bench.py --list 5 || exit 1
tools/gpu_step.sh 200 $out/verify_l20.json python -u tools/verify_bench.py --list 20 --rotate 20 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/verify_bench.py --list 5 > $out/verify_under_rocprof.json 2>&1 || exit 1
