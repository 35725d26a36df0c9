set -o pipefail
mkdir -p gpurun_out/g3
tools/gpu_step.sh 400 gpurun_out/g3/l8.log bash tools/pmc_scale.sh gpurun_out/g3/p 8 fixed:131072:600 cfg2 fixed:32768:2400 fixed:16384:4800 || exit 1
tools/gpu_step.sh 400 gpurun_out/g3/l4.log bash tools/pmc_scale.sh gpurun_out/g3/p 4 fixed:131072:600 cfg2 fixed:32768:2400 || exit 1
