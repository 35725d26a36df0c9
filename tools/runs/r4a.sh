set -o pipefail
# round 4 (a): the round-3 advisor fixes and the honest measurement lines -- -m gpu,
# smoke, driver-form bench with the quota-aware CPU baseline, the self-launched
# --gpus 2 form, cfg3 binned with its traffic, and a rocprof kernel trace of the
# exact driver command (6 streams) beside the serial one.
out=gpurun_out/r4a
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( cat /proc/self/cgroup; cat /sys/fs/cgroup/cpu.max; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))" ) > $out/host.txt 2>&1
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
grep -q "smoke ok" $out/smoke.log || exit 1
tools/gpu_step.sh 300 $out/bench_driver_1.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_gpus2.json python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/cfg3b.json $B --config cfg3 --binned || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/driver_trace -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 > $out/driver_bench.json 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/serial_trace -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 1 --no-cpu-baseline --sustain-ms 0 > $out/serial_bench.json 2>&1 || exit 1
python3 tools/trace_stats.py $out/driver_trace --match "crc32_vring_kernel<3" --skip 1 --out $out/driver_trace_stats.json || exit 1
python3 tools/trace_stats.py $out/serial_trace --match "crc32_vring_kernel<3" --skip 1 --out $out/serial_trace_stats.json || exit 1
echo done > $out/done
