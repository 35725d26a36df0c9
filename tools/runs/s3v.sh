set -o pipefail
# round 2 (session 4): consumer reuses the producer's stage count -- full -m gpu, A/B against the previous build
out=gpurun_out/s3v
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
for r in 1 2 3; do
  tools/gpu_step.sh 200 $out/new_$r.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/old_$r.json python tools/ablib.py tools/libenethip_prev.so bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
