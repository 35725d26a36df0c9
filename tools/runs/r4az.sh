set -o pipefail
# round 4 (az): the binned memory-order diagnostic's parity test
out=gpurun_out/r4az
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread -k "memory_order or records_instance" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
echo done > $out/done
