set -o pipefail
mkdir -p gpurun_out/g16
tools/gpu_step.sh 200 gpurun_out/g16/pipe13.log python -u tools/pipeline.py --path 13 --lanes 8 --depths 1,2,3,4 || exit 1
tools/gpu_step.sh 200 gpurun_out/g16/pipe2.log python -u tools/pipeline.py --path 2 --lanes 8 --depths 1,2,3 || exit 1
