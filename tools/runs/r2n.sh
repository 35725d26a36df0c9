set -o pipefail
# round 2: vring at 64 VGPRs -- parity, pipeline timing, bench (driver form and default)
out=gpurun_out/r2n
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
tools/gpu_step.sh 200 $out/pipe_l4.log python -u tools/pipeline.py --path 0 --lanes 4 --depths 1,2,3,6 || exit 1
tools/gpu_step.sh 200 $out/pipe_l8.log python -u tools/pipeline.py --path 0 --lanes 8 --depths 1,2,3,6 || exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
