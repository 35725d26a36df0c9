set -o pipefail
# round 5 (aa): the batch host entry in place on small / sparse pinned arenas -- harness
# GPU tests, then cfg2 and cfg5 slices, new library against the copy form (r5e), twice
out=gpurun_out/r5aa
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_harness.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2; do
  PCIE_BENCH_SLICES=1 tools/gpu_step.sh 300 $out/slices_new_$rep.log python -u tools/pcie_bench.py 20 || exit 1
  PCIE_BENCH_SLICES=1 ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_r5e.so tools/gpu_step.sh 300 $out/slices_r5e_$rep.log python -u tools/pcie_bench.py 20 || exit 1
done
echo done > $out/done
