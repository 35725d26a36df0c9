set -o pipefail
# round 2: vring with progress-equalizing priority (ablation 1024) vs without
out=gpurun_out/r2k
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in 0 1024 1536; do
  tools/gpu_step.sh 200 $out/pipe_a$a.log python -u tools/pipeline.py --path 0 --lanes 4 --ablate $a --depths 1,6 || exit 1
done
tools/gpu_step.sh 200 $out/pipe_l8_a1024.log python -u tools/pipeline.py --path 0 --lanes 8 --ablate 1024 --depths 1,6 || exit 1
tools/gpu_step.sh 200 $out/tl_prio2.log python -u tools/timeline.py --lanes 4 --path 0 --ablate 1024 || exit 1
