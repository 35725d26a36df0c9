set -o pipefail
# round 5 (c): P = 1 ring with line-aligned windows: policies x fold modes
out=gpurun_out/r5c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/lines.log tools/ringprobe 1200 2 || exit 1
echo done > $out/done
