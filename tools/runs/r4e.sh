set -o pipefail
# round 3 (4e): receive verify (VF): the slot fix-up skips, wave-uniformly, the dwords no lane's slot touches -- verify tests, A/B
out=gpurun_out/r4e
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py -m gpu -v --timeout 240 --timeout-method thread -k "verify" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
cp enet-csharp_amd/libenethip.so ab/libenethip_new.so
for r in 1 2 3; do
  for v in new prev; do
    cp ab/libenethip_$v.so enet-csharp_amd/libenethip.so
    tools/gpu_step.sh 300 $out/verify_${v}_$r.log python -u tools/verify_bench.py --list 20 || exit 1
  done
done
cp ab/libenethip_new.so enet-csharp_amd/libenethip.so
