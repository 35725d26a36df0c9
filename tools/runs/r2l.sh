set -o pipefail
# round 2: vring ring depth 2 / 3 / 4 (ablation 0 / 2048 / 4096), 4 and 8 lanes
out=gpurun_out/r2l
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for l in 4 8; do
for a in 0 2048 4096; do
  tools/gpu_step.sh 200 $out/pipe_l${l}_a$a.log python -u tools/pipeline.py --path 0 --lanes $l --ablate $a --depths 1,6 || exit 1
done
done
