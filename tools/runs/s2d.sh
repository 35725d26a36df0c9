set -o pipefail
# round 2: nontemporal vring stage loads (path 18) vs plain; packet-shaped nt probe
out=gpurun_out/s2d
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_vring.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "vring or empty_groups or list" || exit 1
grep -q " passed" $out/pytest_vring.log || exit 1
grep -q "failed\|Timeout" $out/pytest_vring.log && exit 1
tools/gpu_step.sh 300 $out/streamprobe.txt python -u tools/streamprobe.py all || exit 1
