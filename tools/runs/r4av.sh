set -o pipefail
# round 4 (av): the binned gather at 4 against 8 lanes (default workgroups: two per CU)
out=gpurun_out/r4av
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  tools/gpu_step.sh 300 $out/gather_l8_$rep.log python3 -u tools/gather_bench.py --only gather_binned || exit 1
  tools/gpu_step.sh 300 $out/gather_l4_$rep.log python3 -u tools/gather_bench.py --only gather_binned --lanes 4 || exit 1
done
echo done > $out/done
