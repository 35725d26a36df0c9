set -o pipefail
# round 4 (s): where the waves of a batch-list launch end -- per XCD and per workgroup
out=gpurun_out/r4s
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/timeline_l5_w2_p8.log python -u tools/list_timeline.py 5 2 8 || exit 1
tools/gpu_step.sh 200 $out/timeline_l20_w2_p8.log python -u tools/list_timeline.py 20 2 8 || exit 1
tools/gpu_step.sh 200 $out/timeline_l5_w1_p8.log python -u tools/list_timeline.py 5 1 8 || exit 1
tools/gpu_step.sh 200 $out/timeline_l1_w1_p8.log python -u tools/list_timeline.py 1 1 8 || exit 1
echo done > $out/done
