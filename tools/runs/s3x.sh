set -o pipefail
# round 2 (session 4): the lean / stream kernels' tz correction as unsteps too -- full -m gpu, A/B on the lean paths
out=gpurun_out/s3x
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
for r in 1 2; do
  tools/gpu_step.sh 200 $out/new_cfg3b_$r.json python bench.py --config cfg3 --binned --lanes 4 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/old_cfg3b_$r.json python tools/ablib.py tools/libenethip_prev.so bench.py --config cfg3 --binned --lanes 4 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/new_verify_$r.json python -u tools/verify_bench.py --list 5 || exit 1
  tools/gpu_step.sh 200 $out/old_verify_$r.json python tools/ablib.py tools/libenethip_prev.so tools/verify_bench.py --list 5 || exit 1
  tools/gpu_step.sh 200 $out/new_gather_$r.json python -u tools/gather_bench.py || exit 1
  tools/gpu_step.sh 200 $out/old_gather_$r.json python tools/ablib.py tools/libenethip_prev.so tools/gather_bench.py || exit 1
  tools/gpu_step.sh 200 $out/new_cfg2_$r.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/old_cfg2_$r.json python tools/ablib.py tools/libenethip_prev.so bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
