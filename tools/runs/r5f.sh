set -o pipefail
# round 5 (f): the folders alone: ring kernels with the loader publishing rounds without DMA
out=gpurun_out/r5f
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 120 $out/nodma.log tools/ringprobe 1200 5 || exit 1
echo done > $out/done
