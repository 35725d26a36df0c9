set -o pipefail
# round 2: vring 1 vs 2 workgroups per CU, vs lean
out=gpurun_out/r2e
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/pipe_p0.log python -u tools/pipeline.py --path 0 --lanes 8 --depths 1,6 || exit 1
tools/gpu_step.sh 200 $out/pipe_p0_2wg.log python -u tools/pipeline.py --path 0 --lanes 8 --ablate 512 --depths 1,6 || exit 1
tools/gpu_step.sh 200 $out/pipe_p13.log python -u tools/pipeline.py --path 13 --lanes 8 --depths 1,6 || exit 1
tools/gpu_step.sh 200 $out/pipe_p0_l4.log python -u tools/pipeline.py --path 0 --lanes 4 --depths 1,6 || exit 1
