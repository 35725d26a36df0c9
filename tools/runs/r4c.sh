set -o pipefail
# round 4 (c): the linear kernel after the Horner and direct-fold fixes (parity,
# cfg2 / cfg3 rates, ablations), then the r4a evidence (-m gpu, smoke, driver-form
# bench with the quota-aware CPU baseline, --gpus 2 self-launched, cfg3 binned with
# its traffic, rocprof of the exact driver command).
out=gpurun_out/r4c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest_lin.log python -u -m pytest tests/test_gpu_lin.py -m gpu -v --timeout 120 --timeout-method thread || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/lin22.json $B --path 22 || exit 1
tools/gpu_step.sh 300 $out/lin22_abl1.json $B --path 22 --ablate 2048 || exit 1
tools/gpu_step.sh 300 $out/lin22_cfg3.json $B --path 22 --config cfg3 || exit 1
tools/gpu_step.sh 300 $out/lin22_cfg3_abl1.json $B --path 22 --config cfg3 --ablate 2048 || exit 1
tools/gpu_step.sh 300 $out/lin22_cfg3_abl3.json $B --path 22 --config cfg3 --ablate 6144 || exit 1
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
tools/gpu_step.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh 300 $out/bench_driver_1.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_gpus2.json python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/cfg3b.json $B --config cfg3 --binned || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/driver_trace -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 > $out/driver_bench.json 2>&1 || exit 1
python3 tools/trace_stats.py $out/driver_trace --match "crc32_vring_kernel<3" --skip 1 --out $out/driver_trace_stats.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/serial_trace -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 1 --no-cpu-baseline --sustain-ms 0 > $out/serial_bench.json 2>&1 || exit 1
python3 tools/trace_stats.py $out/serial_trace --match "crc32_vring_kernel<3" --skip 1 --out $out/serial_trace_stats.json || exit 1
echo done > $out/done
