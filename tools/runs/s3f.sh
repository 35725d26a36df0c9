set -o pipefail
# round 2 (session 4): sub-stream probe with the real per-stage costs of a CRC kernel
out=gpurun_out/s3f
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SP_CFGS=56,67,68,35 tools/gpu_step.sh 300 $out/probe.txt python -u tools/streamprobe.py probe || exit 1
