set -o pipefail
# round 4 (aq): cfg3 binned at 8 lanes (one / two workgroups per CU) against 4; the fragment
# reassembly baseline with a kernel trace
out=gpurun_out/r4aq
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --config cfg3 --binned"
for rep in 1 2; do
  tools/gpu_step.sh 300 $out/cfg3b_l4_w1_$rep.json $B --lanes 4 --wgs 1 || exit 1
  tools/gpu_step.sh 300 $out/cfg3b_l8_w1_$rep.json $B --lanes 8 --wgs 1 || exit 1
  tools/gpu_step.sh 300 $out/cfg3b_l8_w2_$rep.json $B --lanes 8 --wgs 2 || exit 1
done
tools/gpu_step.sh 300 $out/frag_1.log python3 -u tools/frag_bench.py || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/frag_trace -o run --output-format csv -- python3 tools/frag_bench.py > $out/frag_trace.log 2>&1 || exit 1
echo done > $out/done
