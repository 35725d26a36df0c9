set -o pipefail
# round 6 (e): the small-batch receive verify read in place over PCIe (csrc/rx_small.hip,
# VERDICT r5 #6): harness tests (every length 6..4096), the GPU suite, the receive call's
# cost at 8-256 DGRAMs against the CPU callback and against the vring verify (path 17),
# and a kernel trace of both
out=gpurun_out/r6e
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest_harness.log python -u -m pytest tests/test_gpu_harness.py -m gpu -v --timeout 180 --timeout-method thread || exit 1
tools/gpu_step.sh 900 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,32,64,128,256 UDP_BENCH_CALL_MODES=gpu,callback,recv \
  tools/gpu_step.sh 300 $out/rx_calls.log python -u tools/udp_bench.py || exit 1
UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,32,64,128,256 UDP_BENCH_CALL_MODES=gpu UDP_BENCH_PATH=17 \
  tools/gpu_step.sh 300 $out/rx_calls_vring.log python -u tools/udp_bench.py || exit 1
UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,256 UDP_BENCH_CALL_MODES=gpu timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d $out/rx_trace -o run --output-format csv -- python3 tools/udp_bench.py > $out/rx_trace.log 2>&1 || exit 1
tools/gpu_step.sh 300 $out/bin_timeline_cold.log python -u tools/bin_timeline.py 3 || exit 1
echo done > $out/done
