set -o pipefail
# round 5 (t): receive verify in place on pinned arenas (no H2D / D2H copies) -- the
# harness GPU tests (pinned and pageable arenas), then the loopback socket rates of the
# new library and of the copy-form library (build_ab/libenethip_r5e.so), interleaved
out=gpurun_out/r5t
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_harness.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2; do
  tools/gpu_step.sh 300 $out/udp_new_$rep.log python -u tools/udp_bench.py || exit 1
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_r5e.so tools/gpu_step.sh 300 $out/udp_copy_$rep.log python -u tools/udp_bench.py || exit 1
done
echo done > $out/done
