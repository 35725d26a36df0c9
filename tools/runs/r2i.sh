set -o pipefail
# round 2: per-wave timeline of the vring kernel (trace instance) and of the lean kernel
out=gpurun_out/r2i
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/tl_vring_l8.log python -u tools/timeline.py --lanes 8 --path 0 || exit 1
tools/gpu_step.sh 200 $out/tl_lean_l8.log python -u tools/timeline.py --lanes 8 --path 13 || exit 1
