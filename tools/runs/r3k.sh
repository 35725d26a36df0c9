set -o pipefail
# round 3 (k): cfg3 binned on the vring records instance by default: GPU suite; SQ counters
# (cfg3 binned, cfg2 lists); no-lookup ablation A/B in order vs tail first; gather kernel
# breakdown; FETCH_SIZE for cfg3 binned and the split cfg5 gather
out=gpurun_out/r3k
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for r in 1 2; do
  tools/gpu_step.sh 300 $out/ab_p0_$r.json $B || exit 1
  tools/gpu_step.sh 300 $out/ab_p21_$r.json $B --path 21 || exit 1
  tools/gpu_step.sh 300 $out/ab_p0_nolook_$r.json $B --ablate 4096 || exit 1
  tools/gpu_step.sh 300 $out/ab_p21_nolook_$r.json $B --path 21 --ablate 4096 || exit 1
done
tools/gpu_step.sh 300 $out/cfg3b_p0.json $B --config cfg3 --binned || exit 1
bash tools/pmc_mix.sh $out/pmc_cfg3b --config cfg3 --binned --reps 8 > $out/pmc_cfg3b.log 2>&1 || exit 1
bash tools/pmc_mix.sh $out/pmc_cfg2 --list 5 --reps 20 > $out/pmc_cfg2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/gather_trace -o run --output-format csv \
  -- python3 tools/gather_bench.py --only gather_binned --reps 20 > $out/gather_trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/cfg3b_fetch -o run --output-format csv \
  -- python3 tools/profile_one.py --config cfg3 --binned --reps 8 --probe > $out/cfg3b_fetch.log 2>&1 || exit 1
python3 tools/traffic_sum.py $out/cfg3b_fetch --bytes 192275835 --calls 8 --probe-bytes 192275824 \
  --what "cfg3 binned (enet_hip_crc32_batch_device_binned, default: vring records, 4 lanes)" --out $out/traffic_cfg3.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/cfg5_fetch -o run --output-format csv \
  -- python3 tools/gather_bench.py --only gather_binned --reps 8 --probe 4 > $out/cfg5_fetch.log 2>&1 || exit 1
python3 tools/traffic_sum.py $out/cfg5_fetch --bytes 274857984 --calls 12 --probe-bytes 274857984 \
  --what "cfg5 binned gather (enet_hip_crc32_gather_binned_device, default: split)" --out $out/traffic_cfg5.json || exit 1
