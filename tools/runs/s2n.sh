set -o pipefail
# round 2: vring ablations: vring stage-load cache policies: default, nt, sc1, sc0 sc1
out=gpurun_out/s2n
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/abl.txt python -u tools/streamprobe.py pol || exit 1
