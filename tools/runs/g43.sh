set -o pipefail
out=gpurun_out/g43
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cfg3 --binned --no-cpu-baseline --steps 100 > $out/cfg3_binned_default.json 2>&1 || exit 1
timeout -k 10 300 python bench.py > $out/bench.json 2>&1 || exit 1
