set -o pipefail
mkdir -p gpurun_out/g9
tools/gpu_step.sh 300 gpurun_out/g9/pytest.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "lean or cfg2 or cfg3 or golden or verify or stream_geometries" || exit 1
tools/gpu_step.sh 120 gpurun_out/g9/tl8.log python -u tools/timeline.py --lanes 8 || exit 1
tools/gpu_step.sh 200 gpurun_out/g9/sweep.log python -u tools/sweep.py --paths 13,14 --lanes 4,8 --wgs 0 --steps 100 --check || exit 1
