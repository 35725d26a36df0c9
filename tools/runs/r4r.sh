set -o pipefail
# round 4 (r): join A/B (global-load join against round 3's flat-load join), then
# round 4 (d)'s sustained-rate set and stream-count bench lines
out=gpurun_out/r4r
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_sel.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_harness.py -k "gather" || exit 1
grep -q " passed" $out/pytest_sel.log && ! grep -q " failed" $out/pytest_sel.log || { echo "parity failed"; exit 1; }
tools/gpu_step.sh 200 $out/gather_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_gather -o run -- python3 -u tools/gather_bench.py --only gather_binned --reps 20 || exit 1
tools/gpu_step.sh 200 $out/gather_prof_r3.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_gather_r3 -o run -- python3 -u tools/gather_bench.py --only gather_binned --reps 20 --ablate 8388608 || exit 1
bash tools/runs/r4d.sh || exit 1
echo done > $out/done
