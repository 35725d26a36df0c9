set -o pipefail
# round 5 (x): the gather host entry on cfg5 slices of growing span (pinned): the new
# library (in place up to 4 MiB), always in place (libenethip_gall), copy form (r5e)
out=gpurun_out/r5x
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for v in new gall r5e; do
    if [ $v = new ]; then unset ENET_HIP_LIBRARY; else export ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so; fi
    PCIE_BENCH_SLICES=1 tools/gpu_step.sh 300 $out/slices_${v}_$rep.log python -u tools/pcie_bench.py 20 || exit 1
  done
done
unset ENET_HIP_LIBRARY
echo done > $out/done
