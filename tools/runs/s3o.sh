set -o pipefail
# round 2 (session 4): fragment copy with 4 chunks per lane in flight -- parity, A/B against the previous build, rocprof split
out=gpurun_out/s3o
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest.log python -u -m pytest tests/test_gpu_fragments.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
for r in 1 2; do
  tools/gpu_step.sh 200 $out/new_$r.txt python -u tools/frag_bench.py || exit 1
  tools/gpu_step.sh 200 $out/old_$r.txt python -u tools/ablib.py tools/libenethip_fragold.so tools/frag_bench.py || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/frag_bench.py > $out/frag_under_rocprof.txt 2>&1 || exit 1
