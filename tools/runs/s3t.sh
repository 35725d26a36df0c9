set -o pipefail
# round 2 (session 4): tz correction by unsteps through the U column (no bit-serial multiply) -- full -m gpu, A/B
out=gpurun_out/s3t
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
for r in 1 2 3; do
  tools/gpu_step.sh 200 $out/new_$r.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/old_$r.json python tools/ablib.py tools/libenethip_mulmod.so bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
tools/gpu_step.sh 200 $out/new_l20.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --list 20 --rotate 20 --streams 1 || exit 1
tools/gpu_step.sh 200 $out/old_l20.json python tools/ablib.py tools/libenethip_mulmod.so bench.py --steps 20 --warmup 5 --no-cpu-baseline --list 20 --rotate 20 --streams 1 || exit 1
tools/gpu_step.sh 200 $out/new_cfg3.json python bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh 200 $out/old_cfg3.json python tools/ablib.py tools/libenethip_mulmod.so bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
