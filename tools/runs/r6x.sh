set -o pipefail
# round 6 (x): the C-ABI from a plain C host (tests/native/c_host.c) on the device
out=gpurun_out/r6x
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ulimit -s > $out/stack_limit.txt
tools/gpu_step.sh 300 $out/pytest_c_host.log python -u -m pytest tests/test_c_host.py -v --timeout 120 --timeout-method thread || exit 1
touch $out/done
