set -o pipefail
# round 4 (aj): cfg3 binned, serial: the scattered out[index] stores priced (ablation 64 =
# 131072: CRCs in record order), with and without the skeleton ablation
out=gpurun_out/r4aj
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --config cfg3 --binned --streams 1"
for rep in 1 2; do
  for a in 0 131072 38912 169984; do
    tools/gpu_step.sh 300 $out/cfg3b_s1_a${a}_$rep.json $B --ablate $a || exit 1
  done
done
echo done > $out/done
