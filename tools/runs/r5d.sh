set -o pipefail
# round 5 (d): P = 4 ring, 12-15 folder waves, line-aligned windows
out=gpurun_out/r5d
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/lines4.log tools/ringprobe 1200 3 || exit 1
echo done > $out/done
