set -o pipefail
# round 2: vring ablations: no lookups, no load in flight during a fold
out=gpurun_out/s2g
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/abl.txt python -u tools/streamprobe.py abl || exit 1
