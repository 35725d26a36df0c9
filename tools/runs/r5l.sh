set -o pipefail
# round 5 (l): the product without the direct / LDS-stream kernels (4 and 8 lanes only;
# the rest in libenethip_diag.so), the one-pass gather join back as the product, the
# split join in diagnostics -- the whole GPU suite, smoke, the default bench command
out=gpurun_out/r5l
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 900 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --steps 20 --warmup 5 || exit 1
echo done > $out/done
