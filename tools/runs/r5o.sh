set -o pipefail
# round 5 (o): the receive pipeline in two halves (submit / complete over two slots) --
# the harness GPU tests, then the loopback socket rates with the new gpu2 mode, twice
out=gpurun_out/r5o
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_harness.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/udp_bench_1.log python -u tools/udp_bench.py || exit 1
tools/gpu_step.sh 300 $out/udp_bench_2.log python -u tools/udp_bench.py || exit 1
for w in 1 2; do
  tools/gpu_step.sh 300 $out/verify_wgs$w.log python -u tools/verify_bench.py --wgs $w --list 20 || exit 1
done
echo done > $out/done
