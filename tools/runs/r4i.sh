set -o pipefail
# round 3 (4i): fragment copy: a round's 16-byte loads issued before its stores (by-value helpers, no LDS-promoted array) -- fragment tests, A/B
out=gpurun_out/r4i
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests/test_gpu_fragments.py -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
cp enet-csharp_amd/libenethip.so ab/libenethip_new.so
for r in 1 2 3; do
  for v in new prev; do
    cp ab/libenethip_$v.so enet-csharp_amd/libenethip.so
    tools/gpu_step.sh 300 $out/frag_${v}_$r.log python -u tools/frag_bench.py || exit 1
  done
done
cp ab/libenethip_new.so enet-csharp_amd/libenethip.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/frag_trace -o run --output-format csv \
  -- python3 tools/frag_bench.py --reps 10 > $out/frag_trace.log 2>&1 || exit 1
