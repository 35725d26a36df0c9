set -o pipefail
# round 5 (b): loader-wave DMA rate by streams per CU x bytes per stream-step; P = 1 ring with default-policy loads
out=gpurun_out/r5b
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/streams.log tools/ringprobe 1200 1 || exit 1
echo done > $out/done
