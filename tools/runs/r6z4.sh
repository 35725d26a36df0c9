set -o pipefail
# round 6: where the single-batch receive verify's time over the checksum goes -- the same
# call with no slot to handle, at one and two workgroups per CU, x2
out=gpurun_out/r6z4
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for w in 2 1; do
    tools/gpu_step.sh 200 $out/verify_w${w}_$rep.log python -u tools/verify_bench.py --list 0 --wgs $w || exit 1
  done
done
touch $out/done
