set -o pipefail
# round 5 (ab): in-place paths restricted to pinned memory of the context's device --
# harness GPU tests, receive per-call costs, cfg2 / cfg5 slices (new library)
out=gpurun_out/r5ab
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_harness.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
UDP_BENCH_CALLS=1 tools/gpu_step.sh 300 $out/calls_new.log python -u tools/udp_bench.py || exit 1
PCIE_BENCH_SLICES=1 tools/gpu_step.sh 300 $out/slices_new.log python -u tools/pcie_bench.py 20 || exit 1
echo done > $out/done
