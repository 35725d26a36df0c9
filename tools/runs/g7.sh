set -o pipefail
mkdir -p gpurun_out/g7
tools/gpu_step.sh 120 gpurun_out/g7/tl8.log python -u tools/timeline.py --lanes 8 || exit 1
tools/gpu_step.sh 120 gpurun_out/g7/dma_tl.log python -u tools/dmabench.py timeline || exit 1
