set -o pipefail
# round 2: full GPU parity after the vring hardening + bench (driver form)
out=gpurun_out/r2m
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
tools/gpu_step.sh 200 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
