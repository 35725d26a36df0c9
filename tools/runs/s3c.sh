set -o pipefail
# round 2 (session 4): line-shaped + nt vring ablations (8 lanes) with the fold on
out=gpurun_out/s3c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/ls.txt python -u tools/streamprobe.py ls || exit 1
