set -o pipefail
mkdir -p gpurun_out/g13
for a in 1 2 3; do
tools/gpu_step.sh 120 gpurun_out/g13/tl_a$a.log python -u tools/timeline.py --lanes 8 --path 13 --ablate $a || exit 1
done
