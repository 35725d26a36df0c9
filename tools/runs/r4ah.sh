set -o pipefail
# round 4 (ah): cfg3 at 4 lanes, serial form: unbinned lists (plain vring instance) against
# the binned records instance, each plain and as its skeleton (2048 + 4096 + 32768)
out=gpurun_out/r4ah
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --config cfg3 --streams 1 --lanes 4"
for rep in 1 2; do
  for a in 0 38912; do
    tools/gpu_step.sh 300 $out/cfg3_list_a${a}_$rep.json $B --ablate $a || exit 1
    tools/gpu_step.sh 300 $out/cfg3_bin_a${a}_$rep.json $B --binned --ablate $a || exit 1
  done
done
echo done > $out/done
