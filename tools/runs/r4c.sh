set -o pipefail
# round 3 (4c): cfg3 binned at 4 (default) vs 8 lanes per packet on the current records instance
out=gpurun_out/r4c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --config cfg3 --binned"
for r in 1 2; do
  tools/gpu_step.sh 300 $out/cfg3b_l4_$r.json $B --lanes 4 || exit 1
  tools/gpu_step.sh 300 $out/cfg3b_l8_$r.json $B --lanes 8 || exit 1
done
