set -o pipefail
# round 2: linear chunk stream with a fold beside it, plain vs nontemporal
out=gpurun_out/s2l
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SP_CFGS=5,7,34,35,36,37 tools/gpu_step.sh 300 $out/probe.txt python -u tools/streamprobe.py probe || exit 1
