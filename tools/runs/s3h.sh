set -o pipefail
# round 2 (session 4): vring lane constants kept live across the ring (no per-iteration
# recompute) -- parity, then A/B against the recompute build on the same box
out=gpurun_out/s3h
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
for r in 1 2; do
  tools/gpu_step.sh 200 $out/new_driver_$r.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/old_driver_$r.json python tools/ablib.py tools/libenethip_lanerecompute.so bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/new_l20_$r.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --list 20 --rotate 20 --streams 1 || exit 1
  tools/gpu_step.sh 200 $out/old_l20_$r.json python tools/ablib.py tools/libenethip_lanerecompute.so bench.py --steps 20 --warmup 5 --no-cpu-baseline --list 20 --rotate 20 --streams 1 || exit 1
done
