set -o pipefail
# round 6 (v): closing evidence of the final build, part 2: rocprof of the serial and of the
# 6-stream driver command, SQ counters, cfg3 / cfg4 / single-batch lines, gather, verify,
# sustained stream, receive-call crossover, fragment reassembly (both decide paths)
out=gpurun_out/r6v
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
sha256sum enet-csharp_amd/libenethip.so > $out/lib_sha.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/serial_trace -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 1 --no-cpu-baseline --sustain-ms 0 > $out/serial_bench.json 2>&1 || exit 1
python3 tools/trace_stats.py $out/serial_trace --match "crc32_vring_kernel<3" --skip 1 --out $out/serial_trace_stats.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/driver_trace -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 > $out/driver_bench.json 2>&1 || exit 1
python3 tools/trace_stats.py $out/driver_trace --match "crc32_vring_kernel<3" --skip 1 --out $out/driver_trace_stats.json || exit 1
bash tools/pmc_mix.sh $out/pmc_cfg2 --list 5 --reps 20 > $out/pmc_cfg2.log 2>&1 || exit 1
python3 tools/pmc_summary.py $out/pmc_cfg2 vring > $out/pmc_cfg2_summary.txt || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/cfg3b_1.json $B --config cfg3 --binned || exit 1
tools/gpu_step.sh 300 $out/cfg3b_serial.json $B --config cfg3 --binned --streams 1 || exit 1
tools/gpu_step.sh 300 $out/cfg4.json $B --config cfg4 || exit 1
tools/gpu_step.sh 300 $out/cfg2_single.json $B --list 0 --streams 1 || exit 1
tools/gpu_step.sh 300 $out/gather_1.log python -u tools/gather_bench.py --only gather_binned || exit 1
tools/gpu_step.sh 300 $out/verify_list20.log python -u tools/verify_bench.py --list 20 || exit 1
tools/gpu_step.sh 300 $out/sustain_vring.log python -u tools/sustain.py --kernel vring --launches 3000 || exit 1
UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,32,64,128,256 UDP_BENCH_CALL_MODES=gpu,callback,recv \
  tools/gpu_step.sh 300 $out/rx_calls.log python -u tools/udp_bench.py || exit 1
tools/gpu_step.sh 300 $out/frag.log python -u tools/frag_bench.py --reps 30 --copy-ref || exit 1
tools/gpu_step.sh 300 $out/frag_w64.log python -u tools/frag_bench.py --reps 30 --words 64 || exit 1
echo done > $out/done
