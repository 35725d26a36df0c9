set -o pipefail
# round 5 (g): ring fold ablations: no masks + no tz multiply (5), no register injection (6), with and without DMA
out=gpurun_out/r5g
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 120 $out/lean.log tools/ringprobe 1200 6 || exit 1
echo done > $out/done
