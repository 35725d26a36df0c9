set -o pipefail
# round 3 (o): host ends re-measured (pipelined host entry with pinned result landing, UDP
# loopback), smoke(), driver-form and default bench lines
out=gpurun_out/r3o
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
grep -q "smoke ok" $out/smoke.log || exit 1
tools/gpu_step.sh 300 $out/pcie_bench.log python -u tools/pcie_bench.py 10 || exit 1
tools/gpu_step.sh 300 $out/udp_bench.log python -u tools/udp_bench.py || exit 1
tools/gpu_step.sh 300 $out/bench_driver_1.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_driver_2.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
tools/gpu_step.sh 300 $out/bench_cfg4.json python bench.py --config cfg4 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
