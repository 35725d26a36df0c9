set -o pipefail
# round 2 (session 3): batch lists on the lean kernel (default) vs the vring kernel -- full gpu suite, list rates, benches
out=gpurun_out/s2s
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/list.txt python -u tools/streamprobe.py list || exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_driver_vring.json python bench.py --gpus 1 --steps 20 --warmup 5 --path 17 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_default_vring.json python bench.py --path 17 --no-cpu-baseline || exit 1
