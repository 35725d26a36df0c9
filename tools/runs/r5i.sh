set -o pipefail
# round 5 (i): A/B of the round-5 library (vring in-place fused fold + interior-stage
# addresses, split gather join) against the round-4 HEAD library, interleaved 3x on
# one box; then the split join against the one-pass join in one (diagnostics) library
out=gpurun_out/r5i
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for v in base r5b; do
    export ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so
    tools/gpu_step.sh 300 $out/bench_${v}_$rep.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    tools/gpu_step.sh 300 $out/cfg3b_${v}_$rep.json python bench.py --config cfg3 --binned --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    tools/gpu_step.sh 300 $out/single_${v}_$rep.json python bench.py --list 0 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    tools/gpu_step.sh 300 $out/verify_${v}_$rep.log python tools/verify_bench.py --list 20 || exit 1
    tools/gpu_step.sh 300 $out/gather_${v}_$rep.log python tools/gather_bench.py --only gather_binned --reps 50 || exit 1
    unset ENET_HIP_LIBRARY
  done
  tools/gpu_step.sh 300 $out/onepass_$rep.log python tools/gather_bench.py --only gather_binned --reps 50 --ablate 4194304 || exit 1
done
tools/gpu_step.sh 300 $out/rocprof_gather.log rocprofv3 --kernel-trace --stats -d $out/prof_gather -o run -- python tools/gather_bench.py --only gather_binned --reps 24 || exit 1
echo done > $out/done
