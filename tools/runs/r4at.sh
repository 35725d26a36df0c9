set -o pipefail
# round 4 (at): fragment reassembly GPU parity with the two-chunk copy
out=gpurun_out/r4at
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "frag" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
echo done > $out/done
