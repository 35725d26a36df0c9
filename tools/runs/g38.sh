set -o pipefail
out=gpurun_out/g38
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "binned or verify or lean" --timeout 120 --timeout-method thread > $out/pytest_binned.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $out/bench.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench2.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cfg3 --lanes 4 --binned --no-cpu-baseline --steps 100 > $out/cfg3_binned_l4.json 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/serial_trace -o run --output-format csv -- python3 bench.py --streams 1 --steps 200 --warmup 20 --no-cpu-baseline > $out/serial_under_rocprof.json 2> $out/serial_under_rocprof.err || exit 1
