set -o pipefail
# round 5 (y): the gather host entry's in-place rule (span <= 4 MiB or segments under 4/5
# of their span): harness GPU tests, then the cfg5 slices twice
out=gpurun_out/r5y
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_harness.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2; do
  PCIE_BENCH_SLICES=1 tools/gpu_step.sh 300 $out/slices_new_$rep.log python -u tools/pcie_bench.py 20 || exit 1
done
UDP_BENCH_SEND_CALLS=1 tools/gpu_step.sh 300 $out/send_new.log python -u tools/udp_bench.py || exit 1
echo done > $out/done
