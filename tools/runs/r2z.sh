set -o pipefail
# round 2: bench defaults = 5-step batch-list launches at 2 workgroups/CU; full GPU suite, driver/default benches, rocprof evidence
out=gpurun_out/r2z
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
tools/gpu_step.sh 300 $out/bench_list0_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 --list 0 --wgs 0 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_list0.json python bench.py --list 0 --wgs 0 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_cfg3.json python bench.py --config cfg3 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_cfg3_binned.json python bench.py --config cfg3 --binned --no-cpu-baseline || exit 1
bash tools/profile_round.sh $out/prof || exit 1
