set -o pipefail
# round 2: line-friendly packet load shapes, plain vs nontemporal
out=gpurun_out/s2e
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SP_CFGS=0,5,7,9,11,14,15,16,17,18,19,20,21,22,23,24,25 tools/gpu_step.sh 300 $out/streamprobe.txt python -u tools/streamprobe.py probe || exit 1
