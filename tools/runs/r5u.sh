set -o pipefail
# round 5 (u): the per-call cost of receive verify on a socket already holding k DGRAMs --
# in place on the pinned arena (new) against the copy form (build_ab/libenethip_r5e.so)
# and the CPU callback, interleaved twice
out=gpurun_out/r5u
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  UDP_BENCH_CALLS=1 tools/gpu_step.sh 300 $out/calls_new_$rep.log python -u tools/udp_bench.py || exit 1
  UDP_BENCH_CALLS=1 ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_r5e.so tools/gpu_step.sh 300 $out/calls_copy_$rep.log python -u tools/udp_bench.py || exit 1
done
echo done > $out/done
