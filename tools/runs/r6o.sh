set -o pipefail
# round 6 (o): workgroups per CU for single large batches: cfg4 (one 1.26 GB batch), one
# cfg4 shard of 8 (131072 packets), the cfg2 single batch; interleaved x2
out=gpurun_out/r6o
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for rep in 1 2; do
  for w in 1 2; do
    tools/gpu_step.sh 300 $out/cfg4_w${w}_$rep.json $B --config cfg4 --wgs $w --streams 1
    tools/gpu_step.sh 300 $out/cfg4s8_w${w}_$rep.json $B --config cfg4 --shard 0/8 --wgs $w --streams 1
    tools/gpu_step.sh 300 $out/cfg4s4_w${w}_$rep.json $B --config cfg4 --shard 0/4 --wgs $w --streams 1
    tools/gpu_step.sh 300 $out/single_w${w}_$rep.json $B --list 0 --wgs $w --streams 1
  done
done
touch $out/done
