set -o pipefail
mkdir -p gpurun_out/g14
tools/gpu_step.sh 120 gpurun_out/g14/tl_a0.log python -u tools/timeline.py --lanes 8 --path 13 || exit 1
