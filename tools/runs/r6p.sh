set -o pipefail
# round 6 (p): the vring kernel's ceiling apart from HBM: the same 5-batch lists from
# HBM, from the Infinity Cache and from L2 (tools/ceiling.py), product and skeleton, 1 and 2 WG/CU
out=gpurun_out/r6p
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in 2 1; do
  tools/gpu_step.sh 240 $out/prod_w$w.log python -u tools/ceiling.py --wgs $w || exit 1
  tools/gpu_step.sh 240 $out/skel_w$w.log python -u tools/ceiling.py --wgs $w --ablation 38912 || exit 1
done
touch $out/done
