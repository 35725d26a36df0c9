set -o pipefail
out=gpurun_out/g30
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
tools/gpu_step.sh 200 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh 300 $out/bench.json python bench.py || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/bench_trace -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --cpu-seconds 2 > $out/bench_under_rocprof.json 2> $out/bench_under_rocprof.err || exit 1
