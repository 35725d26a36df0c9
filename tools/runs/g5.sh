set -o pipefail
mkdir -p gpurun_out/g5
tools/gpu_step.sh 400 gpurun_out/g5/pytest.log python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread || exit 1
tools/gpu_step.sh 200 gpurun_out/g5/sweep.log python -u tools/sweep.py --paths 0,2,13,14 --lanes 4,8 --wgs 0 --steps 100 --check || exit 1
