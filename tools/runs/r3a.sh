set -o pipefail
# round 3 (a): tail-first vring + diag split + wgs parity matrix -- gpu suite, smoke,
# A/B driver-form bench (tail-first path 0 vs in-order path 21), per-kernel rocprof + FETCH_SIZE
out=gpurun_out/r3a
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 900 $out/pytest.log python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED\|Timeout" $out/pytest.log && exit 1
tools/gpu_step.sh 200 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for r in 1 2; do
  tools/gpu_step.sh 300 $out/bench_p0_$r.json python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 2 || exit 1
  tools/gpu_step.sh 300 $out/bench_p21_$r.json python bench.py --gpus 1 --steps 20 --warmup 5 --path 21 --no-cpu-baseline || exit 1
done
bash tools/prof_kernel.sh $out p0_l5 5 || exit 1
bash tools/prof_kernel.sh $out p21_l5 5 --path 21 || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
