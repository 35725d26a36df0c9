set -o pipefail
# round 2 (session 4): final round evidence at HEAD (8 lanes, unstep tz correction, consumer stage count reuse) -- gpu suite, smoke, driver-form and default bench,
# rocprof --stats (default and serial), FETCH_SIZE pass
out=gpurun_out/s3w
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
tools/gpu_step.sh 200 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
tools/gpu_step.sh 300 $out/bench_driver_form.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
bash tools/profile_round.sh $out/prof || exit 1
