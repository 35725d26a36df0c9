set -o pipefail
# round 4 (ac): the binned gather's short-segment bound (join-folded below it, binned above)
out=gpurun_out/r4ac
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_sel.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "short_segment_bounds or gather_binned" || exit 1
grep -q " passed" $out/pytest_sel.log && ! grep -q " failed" $out/pytest_sel.log || { echo "parity failed"; exit 1; }
for rep in 1 2; do
  for b in 0 8 24; do
    tools/gpu_step.sh 200 $out/gather_b${b}_$rep.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_b${b}_$rep -o run -- python3 -u tools/gather_bench.py --only gather_binned --reps 20 --ablate $((16777216 * (1 + b))) || exit 1
  done
  tools/gpu_step.sh 200 $out/gather_b48_$rep.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_b48_$rep -o run -- python3 -u tools/gather_bench.py --only gather_binned --reps 20 || exit 1
done
echo done > $out/done
