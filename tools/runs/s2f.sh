set -o pipefail
# round 2 (session 3): vring ablations -- no edge masks (2048), no lookups (4096), both --
# in 5- and 20-batch lists (streamprobe.py "abl" mode at the time listed exactly these;
# it now lists the s2g / s2i sets)
out=gpurun_out/s2f
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/abl.txt python -u tools/streamprobe.py abl || exit 1
