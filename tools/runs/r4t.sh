set -o pipefail
# round 4 (t): raw per-wave end records of 5-batch lists at 1 and 2 workgroups per CU;
# bench A/B of 1 against 2 workgroups per CU on the product instance
out=gpurun_out/r4t
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export TIMELINE_DUMP=$out/tl
tools/gpu_step.sh 200 $out/timeline_l5_w2_p8.log python -u tools/list_timeline.py 5 2 8 || exit 1
tools/gpu_step.sh 200 $out/timeline_l5_w1_p8.log python -u tools/list_timeline.py 5 1 8 || exit 1
unset TIMELINE_DUMP
B="python bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for w in 1 2; do
  tools/gpu_step.sh 200 $out/cfg2_s1_w$w.json $B --streams 1 --wgs $w || exit 1
  tools/gpu_step.sh 200 $out/cfg2_s6_w$w.json $B --wgs $w || exit 1
done
for w in 2 1; do
  tools/gpu_step.sh 200 $out/cfg2_s1_w${w}_b.json $B --streams 1 --wgs $w || exit 1
  tools/gpu_step.sh 200 $out/cfg2_s6_w${w}_b.json $B --wgs $w || exit 1
done
echo done > $out/done
