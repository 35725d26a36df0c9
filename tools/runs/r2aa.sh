set -o pipefail
# round 2: metadata-branch wait counts the 3 DMA loads (vmcnt 5); parity, benches, rocprof evidence
out=gpurun_out/r2aa
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/listprobe.log python -u tools/listprobe.py || exit 1
grep -q "^done" $out/listprobe.log || exit 1
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
tools/gpu_step.sh 300 $out/bench_list0.json python bench.py --list 0 --wgs 0 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_list0_s1.json python bench.py --list 0 --wgs 0 --streams 1 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_l8.json python bench.py --lanes 8 --no-cpu-baseline || exit 1
bash tools/profile_round.sh $out/prof || exit 1
