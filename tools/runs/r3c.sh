set -o pipefail
# round 3 (c): stress for intermittent wrong CRCs (vring at 1 / 2 workgroups per CU); GPU suite
out=gpurun_out/r3c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/stress.log python -u tools/dbg/stress.py 25 || exit 1
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
tools/gpu_step.sh 300 $out/pcie_bench.log python -u tools/pcie_bench.py 10 || exit 1
tools/gpu_step.sh 300 $out/udp_bench.log python -u tools/udp_bench.py || exit 1
tools/gpu_step.sh 120 $out/sustain_probe.log python -u tools/sustain.py --kernel probe --launches 3000 || exit 1
tools/gpu_step.sh 120 $out/sustain_vring.log python -u tools/sustain.py --kernel vring --launches 3000 || exit 1
