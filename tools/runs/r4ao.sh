set -o pipefail
# round 4 (ao): range coder at 16 lanes per wave x 16 waves per CU (the new default):
# parity (incl. the lanes/waves knobs), then rc_bench default x2
out=gpurun_out/r4ao
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests/test_gpu_range_coder.py -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/rc_1.log python3 -u tools/rc_bench.py || exit 1
tools/gpu_step.sh 300 $out/rc_2.log python3 -u tools/rc_bench.py || exit 1
echo done > $out/done
