set -o pipefail
# round 2: vring without spills, 1 vs 2 workgroups per CU, 4 vs 8 lanes
out=gpurun_out/r2f
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for l in 8 4; do
  tools/gpu_step.sh 200 $out/pipe_l${l}.log python -u tools/pipeline.py --path 0 --lanes $l --depths 1,2,6 || exit 1
  tools/gpu_step.sh 200 $out/pipe_l${l}_2wg.log python -u tools/pipeline.py --path 0 --lanes $l --ablate 512 --depths 1,2,6 || exit 1
done
