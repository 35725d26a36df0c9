set -o pipefail
# round 3 (4a): the gather join fills its 4 KiB slicing-by-4 tables by rows (two 16-B loads per thread) -- gather tests, A/B
out=gpurun_out/r4a
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py -m gpu -v --timeout 240 --timeout-method thread -k "gather" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
cp enet-csharp_amd/libenethip.so ab/libenethip_new.so
for r in 1 2 3; do
  for v in new prev; do
    cp ab/libenethip_$v.so enet-csharp_amd/libenethip.so
    tools/gpu_step.sh 300 $out/gather_${v}_$r.log python -u tools/gather_bench.py --only gather_binned || exit 1
  done
done
cp ab/libenethip_new.so enet-csharp_amd/libenethip.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/gather_trace -o run --output-format csv \
  -- python3 tools/gather_bench.py --only gather_binned --reps 20 > $out/gather_trace.log 2>&1 || exit 1
