set -o pipefail
# round 2 (session 4): sub-stream access shapes with a fold (linear-stream CRC design)
out=gpurun_out/s3a
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SP_CFGS=7,24,35,41,54,55,56,57,58,59,60,61,62,63,64,65,66 tools/gpu_step.sh 300 $out/probe.txt python -u tools/streamprobe.py probe || exit 1
