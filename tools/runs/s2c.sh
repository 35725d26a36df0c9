set -o pipefail
# round 2: long-stream read rate per access shape; vring rate vs batch-list length
out=gpurun_out/s2c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/streamprobe.txt python -u tools/streamprobe.py all || exit 1
