set -o pipefail
# round 2 (session 3): one 1.57 GB batch per launch -- vring vs lean streaming rates without per-launch start/drain
out=gpurun_out/s2r
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/big.txt python -u tools/streamprobe.py big || exit 1
