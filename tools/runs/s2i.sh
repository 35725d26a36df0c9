set -o pipefail
# round 2: vring ablations: skeleton ablation (no masks, lookups, corrections)
out=gpurun_out/s2i
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/abl.txt python -u tools/streamprobe.py abl || exit 1
SP_CFGS=9,11,14,16,18 tools/gpu_step.sh 300 $out/probe.txt python -u tools/streamprobe.py probe || exit 1
