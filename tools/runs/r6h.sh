set -o pipefail
# round 6 (h): workgroups per CU after the round-6 changes, interleaved x3 on one box: cfg2
# 5-batch lists (serial and driver form) and cfg3 binned (the compact records instance at two)
out=gpurun_out/r6h
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2 3; do
  for w in 1 2; do
    tools/gpu_step.sh 300 $out/cfg2_ser_w${w}_$rep.json $B --wgs $w --streams 1 --sustain-ms 0 || exit 1
    tools/gpu_step.sh 300 $out/cfg2_drv_w${w}_$rep.json $B --wgs $w || exit 1
    tools/gpu_step.sh 300 $out/cfg3b_ser_w${w}_$rep.json $B --wgs $w --config cfg3 --binned --streams 1 --sustain-ms 0 || exit 1
  done
done
echo done > $out/done
