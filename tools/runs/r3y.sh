set -o pipefail
# round 3 (y): records instance: tz mod 8 by small x^(-8c) tables (no conflicted unsteps) -- tests, A/B vs the previous library
# previous library (ab/libenethip_prev.so swapped in place), interleaved
out=gpurun_out/r3y
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
cp enet-csharp_amd/libenethip.so ab/libenethip_new.so
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for r in 1 2; do
  for v in new prev; do
    cp ab/libenethip_$v.so enet-csharp_amd/libenethip.so
    tools/gpu_step.sh 300 $out/cfg3b_${v}_$r.json $B --config cfg3 --binned || exit 1
    tools/gpu_step.sh 300 $out/cfg2_${v}_$r.json $B || exit 1
    tools/gpu_step.sh 300 $out/gather_${v}_$r.log python -u tools/gather_bench.py --only gather_binned || exit 1
  done
done
cp ab/libenethip_new.so enet-csharp_amd/libenethip.so
