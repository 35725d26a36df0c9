set -o pipefail
# round 3 (u): load-only probe of the packet shapes at 1/2/4/8 lanes per packet, in order and shuffled
out=gpurun_out/r3u
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 120 $out/alignprobe.log tools/alignprobe || exit 1
