set -o pipefail
# round 3 (q): split join on a side stream (prep concurrent with the checksum pass), wave-scan bin kernel, BIN index stash (lane constants live)
out=gpurun_out/r3q
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest_gather.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py -m gpu -v --timeout 240 --timeout-method thread -k "gather or binned or bin" || exit 1
grep -q " passed" $out/pytest_gather.log || exit 1
grep -q "FAILED" $out/pytest_gather.log && exit 1
for r in 1 2 3; do
  tools/gpu_step.sh 300 $out/gather_$r.log python -u tools/gather_bench.py --only gather_binned || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/gather_trace -o run --output-format csv \
  -- python3 tools/gather_bench.py --only gather_binned --reps 20 > $out/gather_trace.log 2>&1 || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/cfg3b_1.json $B --config cfg3 --binned || exit 1
tools/gpu_step.sh 300 $out/cfg3b_2.json $B --config cfg3 --binned || exit 1
