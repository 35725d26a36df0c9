set -o pipefail
# round 5 (s): A/B of nt loads on the vring's interior stages (ENET_HIP_NT_INNER build,
# libenethip_ntin) against the product library (r5e), interleaved 3x on one box
out=gpurun_out/r5s
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for v in r5e ntin; do
    export ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so
    tools/gpu_step.sh 300 $out/bench_${v}_$rep.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    tools/gpu_step.sh 300 $out/cfg3b_${v}_$rep.json python bench.py --config cfg3 --binned --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    tools/gpu_step.sh 300 $out/single_${v}_$rep.json python bench.py --list 0 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    tools/gpu_step.sh 300 $out/verify_${v}_$rep.log python tools/verify_bench.py --list 20 || exit 1
    unset ENET_HIP_LIBRARY
  done
done
echo done > $out/done
