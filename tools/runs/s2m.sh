set -o pipefail
# round 2: packet folds with exec-masked (not zero-line) out-of-window pieces
out=gpurun_out/s2m
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SP_CFGS=28,30,38,39,40,41 tools/gpu_step.sh 300 $out/probe.txt python -u tools/streamprobe.py probe || exit 1
