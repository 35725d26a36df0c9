set -o pipefail
# round 4 (au): the full GPU suite, smoke and the driver-form bench at HEAD (after the range
# coder and fragment copy changes)
out=gpurun_out/r4au
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
grep -q "smoke ok" $out/smoke.log || exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/rc.log python3 -u tools/rc_bench.py || exit 1
tools/gpu_step.sh 300 $out/frag.log python3 -u tools/frag_bench.py || exit 1
echo done > $out/done
