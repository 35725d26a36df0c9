set -o pipefail
# round 5 (ai): the group-end corrections trimmed (packed correction columns; one test for
# the tz steps below 16) -- the full GPU suite on the new library, cfg2 VALU counts of both,
# and a short A/B against r5f
out=gpurun_out/r5ai
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 900 $out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" $out/pytest_gpu.log || exit 1
grep -qE "failed|FAILED|error" $out/pytest_gpu.log && exit 1
for v in r5f tzc; do
  export ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so
  bash tools/pmc_mix.sh $out/pmc_cfg2_$v --list 5 --reps 20 > $out/pmc_cfg2_$v.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $out/pmc_cfg2_$v vring > $out/pmc_cfg2_${v}_summary.txt || exit 1
  unset ENET_HIP_LIBRARY
done
for rep in 1 2; do
  for v in r5f tzc; do
    export ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so
    tools/gpu_step.sh 300 $out/bench_${v}_$rep.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    tools/gpu_step.sh 300 $out/cfg3b_${v}_$rep.json python bench.py --config cfg3 --binned --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    tools/gpu_step.sh 300 $out/verify_${v}_$rep.log python tools/verify_bench.py --list 20 || exit 1
    unset ENET_HIP_LIBRARY
  done
done
echo done > $out/done
