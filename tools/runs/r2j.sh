set -o pipefail
# round 2: fragment overlap fix (deferred serial pass) parity + cfg5 timing; vring timeline by wave slot
out=gpurun_out/r2j
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_frag.log python -u -m pytest tests/test_gpu_fragments.py -x -v --timeout 120 --timeout-method thread || exit 1
tools/gpu_step.sh 200 $out/frag_bench.log python -u tools/frag_bench.py || exit 1
tools/gpu_step.sh 200 $out/tl_vring_l8.log python -u tools/timeline.py --lanes 8 --path 0 || exit 1
tools/gpu_step.sh 200 $out/tl_vring_l4.log python -u tools/timeline.py --lanes 4 --path 0 || exit 1
