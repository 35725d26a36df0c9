set -o pipefail
# round 6 (q): line-shaped stage loads (ablation 16384: 128-B windows, each instruction one
# whole line per packet, the fold intact but its tables not repositioned -- WRONG CRCs)
# with the current fold, default and nt policy, against the product on the same box
out=gpurun_out/r6q
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="python -u tools/ceiling.py --levels hbm"
for rep in 1 2; do
  for w in 2 1; do
    tools/gpu_step.sh 200 $out/prod_w${w}_$rep.log $C --wgs $w || exit 1
    tools/gpu_step.sh 200 $out/line_w${w}_$rep.log $C --wgs $w --path 17 --ablation 16384 || exit 1
    tools/gpu_step.sh 200 $out/linent_w${w}_$rep.log $C --wgs $w --path 18 --ablation 16384 || exit 1
    tools/gpu_step.sh 200 $out/lineskelnt_w${w}_$rep.log $C --wgs $w --path 18 --ablation 55296 || exit 1
    tools/gpu_step.sh 200 $out/skel_w${w}_$rep.log $C --wgs $w --ablation 38912 || exit 1
  done
done
touch $out/done
