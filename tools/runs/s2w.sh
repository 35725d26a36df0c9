set -o pipefail
# round 2 (session 3): per-wave end-time spread inside one vring batch-list launch (static deal)
out=gpurun_out/s2w
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/tl_l20_w2.txt python -u tools/list_timeline.py 20 2 || exit 1
tools/gpu_step.sh 200 $out/tl_l5_w2.txt python -u tools/list_timeline.py 5 2 || exit 1
tools/gpu_step.sh 200 $out/tl_l20_w1.txt python -u tools/list_timeline.py 20 1 || exit 1
