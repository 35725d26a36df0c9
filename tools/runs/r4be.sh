set -o pipefail
# round 4 (be): the full GPU suite and smoke at HEAD (after the fragment descriptors change)
out=gpurun_out/r4be
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
tools/gpu_step.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
grep -q "smoke ok" $out/smoke.log || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
echo done > $out/done
