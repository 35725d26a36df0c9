set -o pipefail
# round 4 (ak): cfg3 binned, serial: the records instance on records left in memory order
# (diagnostics 2^30) against the binned order, plain and as the skeleton (38912)
out=gpurun_out/r4ak
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --config cfg3 --binned --streams 1"
for rep in 1 2; do
  for a in 0 1073741824 38912 1073780736; do
    tools/gpu_step.sh 300 $out/cfg3b_s1_a${a}_$rep.json $B --ablate $a || exit 1
  done
done
echo done > $out/done
