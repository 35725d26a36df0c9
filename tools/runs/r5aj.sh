set -o pipefail
# round 5 (aj): loopback receive with 1, 2 and 4 sender threads, so that the receiver rather
# than the sender bounds the rate: recv alone, the GPU (sync and two-slot, in place) and the
# CPU callback
out=gpurun_out/r5aj
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 1 2 4; do
  UDP_BENCH_SENDERS=$n UDP_BENCH_RECV_MODES=recv,gpu,gpu2,callback tools/gpu_step.sh 300 $out/recv_s$n.log python -u tools/udp_bench.py || exit 1
done
UDP_BENCH_SENDERS=4 UDP_BENCH_RECV_MODES=recv,gpu,gpu2,callback tools/gpu_step.sh 300 $out/recv_s4_b.log python -u tools/udp_bench.py || exit 1
echo done > $out/done
