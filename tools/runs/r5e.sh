set -o pipefail
# round 5 (e): P = 4 ring with LDS handshake words instead of per-round barriers
out=gpurun_out/r5e
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 120 $out/hs4.log tools/ringprobe 1200 4 || exit 1
echo done > $out/done
