set -o pipefail
# round 3 (s): records instance with end-aligned windows (EA), BIN index stash, wave-scan bin kernel; full -m gpu
out=gpurun_out/r3s
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for r in 1 2; do
  tools/gpu_step.sh 300 $out/gather_$r.log python -u tools/gather_bench.py --only gather_binned || exit 1
done
tools/gpu_step.sh 300 $out/gather_l4.log python -u tools/gather_bench.py --only gather_binned --lanes 4 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/gather_trace -o run --output-format csv \
  -- python3 tools/gather_bench.py --only gather_binned --reps 20 > $out/gather_trace.log 2>&1 || exit 1
tools/gpu_step.sh 120 $out/alignprobe.log tools/alignprobe || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/cfg3b_1.json $B --config cfg3 --binned || exit 1
tools/gpu_step.sh 300 $out/cfg3b_2.json $B --config cfg3 --binned || exit 1
tools/gpu_step.sh 300 $out/cfg2_1.json $B || exit 1
