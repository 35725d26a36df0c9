set -o pipefail
# round 3 (h): in-order product default + zero-byte multiplier tables (tz) + asm slot counter:
# GPU suite, A/B benches (lists at 1 / 2 workgroups per CU, single-batch launches), verify, rocprof + FETCH
out=gpurun_out/r3h
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for r in 1 2; do
  for w in 2 1; do
    tools/gpu_step.sh 300 $out/bench_p0_w${w}_$r.json python bench.py --gpus 1 --steps 20 --warmup 5 --wgs $w --no-cpu-baseline --sustain-ms 0 || exit 1
    tools/gpu_step.sh 300 $out/bench_single_w${w}_$r.json python bench.py --gpus 1 --steps 20 --warmup 5 --wgs $w --list 0 --no-cpu-baseline --sustain-ms 0 || exit 1
  done
done
tools/gpu_step.sh 300 $out/bench_p21_w2.json python bench.py --gpus 1 --steps 20 --warmup 5 --path 21 --no-cpu-baseline --sustain-ms 0 || exit 1
tools/gpu_step.sh 300 $out/verify_bench.log python -u tools/verify_bench.py --list 20 || exit 1
tools/gpu_step.sh 300 $out/verify_bench_l5.log python -u tools/verify_bench.py --list 5 || exit 1
bash tools/prof_kernel.sh $out p0_w2 5 --wgs 2 || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
