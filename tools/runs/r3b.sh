set -o pipefail
# round 3 (b): debug the walk path at two workgroups per CU; then the full GPU suite without -x
out=gpurun_out/r3b
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/walk_dbg.log python -u tools/dbg/walk_dbg.py || exit 1
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
