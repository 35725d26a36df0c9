set -o pipefail
# round 5 (q): cfg5 binned gather at 4 lanes (128-byte stages: 11 for a 1376-byte window,
# 2 % padding) against the default 8 (256-byte stages: 6, 10 % padding), interleaved 3x
out=gpurun_out/r5q
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for l in 8 4; do
    tools/gpu_step.sh 300 $out/gather_l${l}_$rep.log python -u tools/gather_bench.py --only gather_binned --lanes $l --reps 50 || exit 1
  done
  tools/gpu_step.sh 300 $out/gather_l4_w1_$rep.log python -u tools/gather_bench.py --only gather_binned --lanes 4 --wgs 1 --reps 50 || exit 1
done
echo done > $out/done
