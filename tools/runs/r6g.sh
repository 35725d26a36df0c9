set -o pipefail
# round 6 (g): kernel traces of the PCIe probe (the same clock as the receive kernels' traces),
# and the single-batch cfg2 timeline
out=gpurun_out/r6g
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/probe_trace -o run --output-format csv -- ./tools/pcieprobe > $out/pcieprobe.log 2>&1 || exit 1
tools/gpu_step.sh 300 $out/timeline_single_w1.log python -u tools/list_timeline.py 1 1 8 || exit 1
tools/gpu_step.sh 300 $out/timeline_single_w2.log python -u tools/list_timeline.py 1 2 8 || exit 1
tools/gpu_step.sh 300 $out/timeline_list5_w2.log python -u tools/list_timeline.py 5 2 8 || exit 1
tools/gpu_step.sh 600 $out/pytest_harness.log python -u -m pytest tests/test_gpu_harness.py -m gpu -v --timeout 180 --timeout-method thread || exit 1
for rep in 1 2; do
  UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,64,256 UDP_BENCH_CALL_MODES=gpu,callback \
    tools/gpu_step.sh 300 $out/rx_new_$rep.log python -u tools/udp_bench.py || exit 1
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_rxs1.so UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,64,256 UDP_BENCH_CALL_MODES=gpu \
    tools/gpu_step.sh 300 $out/rx_rxs1_$rep.log python -u tools/udp_bench.py || exit 1
  UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,64,256 UDP_BENCH_CALL_MODES=gpu UDP_BENCH_PATH=17 \
    tools/gpu_step.sh 300 $out/rx_vring_$rep.log python -u tools/udp_bench.py || exit 1
done
UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,256 UDP_BENCH_CALL_MODES=gpu timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d $out/rx_trace -o run --output-format csv -- python3 tools/udp_bench.py > $out/rx_trace.log 2>&1 || exit 1
echo done > $out/done
