set -o pipefail
# round 2 (session 4): 4 vs 8 lanes per packet, interleaved repeats (driver form and serial 5-batch region)
out=gpurun_out/s3k
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do for l in 4 8; do
  tools/gpu_step.sh 200 $out/l${l}_r${r}.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --lanes $l || exit 1
  tools/gpu_step.sh 200 $out/l${l}_s60_r${r}.json python bench.py --steps 60 --warmup 5 --no-cpu-baseline --lanes $l || exit 1
done; done
