set -o pipefail
# round 4 (y): single-batch checksum / verify at 1 and 2 workgroups per CU
out=gpurun_out/r4y
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for w in 1 2; do
    tools/gpu_step.sh 300 $out/verify_w${w}_$rep.log python3 -u tools/verify_bench.py --reps 50 --list 5 --wgs $w || exit 1
  done
done
echo done > $out/done
