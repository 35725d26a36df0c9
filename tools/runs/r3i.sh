set -o pipefail
# round 3 (i): where cfg3 (binned / unbinned), the cfg5 gather and the serial cfg2 bench stand;
# FETCH_SIZE passes for cfg3 binned and the cfg5 binned gather; rocprof of the serial bench command
out=gpurun_out/r3i
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/cfg3b_p0.json $B --config cfg3 --binned || exit 1
for l in 4 8; do for w in 1 2; do
  tools/gpu_step.sh 300 $out/cfg3b_p17_l${l}_w${w}.json $B --config cfg3 --binned --path 17 --lanes $l --wgs $w || exit 1
done; done
tools/gpu_step.sh 300 $out/cfg3_p0.json $B --config cfg3 || exit 1
tools/gpu_step.sh 300 $out/cfg3_p0_l4.json $B --config cfg3 --lanes 4 || exit 1
tools/gpu_step.sh 300 $out/gather_p0.log python -u tools/gather_bench.py || exit 1
tools/gpu_step.sh 300 $out/gather_p17_l4.log python -u tools/gather_bench.py --path 17 --lanes 4 --only gather_binned || exit 1
tools/gpu_step.sh 300 $out/gather_p17_l8.log python -u tools/gather_bench.py --path 17 --lanes 8 --only gather_binned || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/cfg3b_fetch -o run --output-format csv \
  -- python3 tools/profile_one.py --config cfg3 --binned --reps 8 --probe > $out/cfg3b_fetch.log 2>&1 || exit 1
python3 tools/traffic_sum.py $out/cfg3b_fetch --bytes 192275835 --calls 8 --probe-bytes 192275824 \
  --what "cfg3 binned (enet_hip_crc32_batch_device_binned, path 0)" --out $out/traffic_cfg3.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/cfg5_fetch -o run --output-format csv \
  -- python3 tools/gather_bench.py --only gather_binned --reps 8 --probe 4 > $out/cfg5_fetch.log 2>&1 || exit 1
python3 tools/traffic_sum.py $out/cfg5_fetch --bytes 274857984 --calls 12 --probe-bytes 274857984 \
  --what "cfg5 binned gather (enet_hip_crc32_gather_binned_device, path 0)" --out $out/traffic_cfg5.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/serial_trace -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 1 --no-cpu-baseline --sustain-ms 0 > $out/serial_bench.json 2>&1 || exit 1
python3 tools/trace_stats.py $out/serial_trace --match "crc32_vring_kernel<3" > $out/serial_trace_all.json
