set -o pipefail
out=gpurun_out/g35
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k binned --timeout 120 --timeout-method thread > $out/pytest_binned.log 2>&1 || exit 1
for l in 4 8; do
  timeout -k 10 200 python bench.py --config cfg3 --lanes $l --binned --no-cpu-baseline --steps 100 > $out/cfg3_binned_l$l.json 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/cfg3_binned_l${l}_trace -o run --output-format csv -- python3 bench.py --config cfg3 --lanes $l --binned --streams 1 --steps 100 --no-cpu-baseline > $out/cfg3_binned_l${l}_serial_rocprof.json 2> $out/cfg3_binned_l${l}_rocprof.err || exit 1
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
