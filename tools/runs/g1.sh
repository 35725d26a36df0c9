set -o pipefail
mkdir -p gpurun_out/g1
tools/gpu_step.sh 300 gpurun_out/g1/pytest.log python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread || exit 1
tools/gpu_step.sh 200 gpurun_out/g1/bench.log python -u bench.py --cpu-seconds 3 || exit 1
tools/gpu_step.sh 300 gpurun_out/g1/sweep.log python -u tools/sweep.py --paths 0,2,3,4,5,6,7,8,9,10,11,12 --lanes 4,8,16 --wgs 0 --steps 100 || exit 1
