set -o pipefail
# round 3 (w): cfg4 (one 1.26 GB batch per launch) at 1 vs 2 workgroups per CU
out=gpurun_out/r3w
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --config cfg4"
for r in 1 2; do
  tools/gpu_step.sh 300 $out/cfg4_w1_$r.json $B --wgs 1 || exit 1
  tools/gpu_step.sh 300 $out/cfg4_w2_$r.json $B --wgs 2 || exit 1
done
B2="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --list 0"
for r in 1 2; do
  tools/gpu_step.sh 300 $out/cfg2_l0_w1_$r.json $B2 --wgs 1 || exit 1
  tools/gpu_step.sh 300 $out/cfg2_l0_w2_$r.json $B2 --wgs 2 || exit 1
done
