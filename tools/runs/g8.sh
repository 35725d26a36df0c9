set -o pipefail
mkdir -p gpurun_out/g8
tools/gpu_step.sh 120 gpurun_out/g8/tl8.log python -u tools/timeline.py --lanes 8 || exit 1
tools/gpu_step.sh 120 gpurun_out/g8/tl4.log python -u tools/timeline.py --lanes 4 || exit 1
