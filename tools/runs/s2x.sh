set -o pipefail
# round 2 (session 3): vring with per-workgroup dynamic slots -- full gpu suite, wave end spread, list rates, benches
out=gpurun_out/s2x
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
tools/gpu_step.sh 200 $out/tl_l20_w2.txt python -u tools/list_timeline.py 20 2 || exit 1
tools/gpu_step.sh 200 $out/tl_l20_w1.txt python -u tools/list_timeline.py 20 1 || exit 1
tools/gpu_step.sh 300 $out/list.txt python -u tools/streamprobe.py list || exit 1
tools/gpu_step.sh 200 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 200 $out/bench_driver_l20.json python bench.py --gpus 1 --steps 20 --warmup 5 --list 20 --rotate 20 --streams 1 --no-cpu-baseline || exit 1
tools/gpu_step.sh 200 $out/bench_driver_wgs1.json python bench.py --gpus 1 --steps 20 --warmup 5 --wgs 1 --no-cpu-baseline || exit 1
tools/gpu_step.sh 200 $out/bench_default.json python bench.py --no-cpu-baseline || exit 1
