set -o pipefail
# round 6: the produce step at s_setprio 3 (diagnostics instance, ablation 65536 at 8 lanes)
# against the product, interleaved x3, 5-batch lists from HBM (tools/ceiling.py)
out=gpurun_out/r6z3
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="python -u tools/ceiling.py --levels hbm,l2"
for rep in 1 2 3; do
  tools/gpu_step.sh 200 $out/prod_$rep.log $C --wgs 2 || exit 1
  tools/gpu_step.sh 200 $out/prio_$rep.log $C --wgs 2 --path 17 --ablation 65536 || exit 1
done
touch $out/done
