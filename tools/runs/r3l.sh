set -o pipefail
# round 3 (l): binned gather without global atomics (padded tiles + tile counts read by the
# vring records instance) and a join that loads small segments first (slicing-by-4):
# GPU suite, gather benches, kernel breakdown, FETCH_SIZE
out=gpurun_out/r3l
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/gather_l8.log python -u tools/gather_bench.py --only gather_binned || exit 1
tools/gpu_step.sh 300 $out/gather_l4.log python -u tools/gather_bench.py --only gather_binned --lanes 4 || exit 1
tools/gpu_step.sh 300 $out/gather_l8_b.log python -u tools/gather_bench.py --only gather_binned || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/gather_trace -o run --output-format csv \
  -- python3 tools/gather_bench.py --only gather_binned --reps 20 > $out/gather_trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/cfg5_fetch -o run --output-format csv \
  -- python3 tools/gather_bench.py --only gather_binned --reps 8 --probe 4 > $out/cfg5_fetch.log 2>&1 || exit 1
python3 tools/traffic_sum.py $out/cfg5_fetch --bytes 274857984 --calls 12 --probe-bytes 274857984 \
  --what "cfg5 binned gather (enet_hip_crc32_gather_binned_device, default: split, tile counts)" --out $out/traffic_cfg5.json || exit 1
