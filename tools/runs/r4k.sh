set -o pipefail
# round 3 (4k): last validation at HEAD -- -m gpu, smoke, driver-form bench, cfg3 binned, gather, verify lists
out=gpurun_out/r4k
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
grep -q "smoke ok" $out/smoke.log || exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/cfg3b.json $B --config cfg3 --binned || exit 1
tools/gpu_step.sh 300 $out/gather.log python -u tools/gather_bench.py --only gather_binned || exit 1
tools/gpu_step.sh 300 $out/verify_list20.log python -u tools/verify_bench.py --list 20 || exit 1
