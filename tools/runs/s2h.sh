set -o pipefail
# round 2: vring ablations: 8 lanes, line-shaped loads + 128-B windows (memory side)
out=gpurun_out/s2h
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/abl.txt python -u tools/streamprobe.py abl8 || exit 1
