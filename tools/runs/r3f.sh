set -o pipefail
# round 3 (f): tail-first (path 0) vs in-order (path 21) A/B, 1 and 2 workgroups per CU;
# per-kernel rocprof + FETCH_SIZE for both at 2 workgroups per CU
out=${OUT:-gpurun_out/r3f}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for w in 2 1; do
    tools/gpu_step.sh 300 $out/bench_p0_w${w}_$r.json python bench.py --gpus 1 --steps 20 --warmup 5 --wgs $w --no-cpu-baseline --sustain-ms 0 || exit 1
    tools/gpu_step.sh 300 $out/bench_p21_w${w}_$r.json python bench.py --gpus 1 --steps 20 --warmup 5 --wgs $w --path 21 --no-cpu-baseline --sustain-ms 0 || exit 1
  done
done
bash tools/prof_kernel.sh $out p0_w2 5 --wgs 2 || exit 1
bash tools/prof_kernel.sh $out p21_w2 5 --wgs 2 --path 21 || exit 1
bash tools/prof_kernel.sh $out p0_w1 5 --wgs 1 || exit 1
