set -o pipefail
# round 5 (w): the gather host entry in place on pinned arenas -- harness GPU tests, then
# the per-call stamp + send cost: new library (in place up to 4 MiB of span), always in
# place (build_ab/libenethip_gall.so), copy form (build_ab/libenethip_r5e.so)
out=gpurun_out/r5w
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_harness.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2; do
  UDP_BENCH_SEND_CALLS=1 tools/gpu_step.sh 300 $out/send_new_$rep.log python -u tools/udp_bench.py || exit 1
  UDP_BENCH_SEND_CALLS=1 ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_gall.so tools/gpu_step.sh 300 $out/send_all_$rep.log python -u tools/udp_bench.py || exit 1
  UDP_BENCH_SEND_CALLS=1 ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_r5e.so tools/gpu_step.sh 300 $out/send_copy_$rep.log python -u tools/udp_bench.py || exit 1
done
echo done > $out/done
