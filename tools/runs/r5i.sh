set -o pipefail
# round 5 (i): the split gather join (pre-join beside the binning tiles, post-join per
# segment) -- gather parity, the compressed UDP pipelines, the fragment slots-path
# threshold; then cfg5 A/B against the one-pass join (diagnostics 4194304) and rocprof
out=gpurun_out/r5i
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread -k "gather or harness or fragments" tests/test_gpu_parity.py tests/test_gpu_harness.py tests/test_gpu_fragments.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2 3; do
  tools/gpu_step.sh 300 $out/split_$rep.json python tools/gather_bench.py --only gather_binned --reps 50 || exit 1
  tools/gpu_step.sh 300 $out/onepass_$rep.json python tools/gather_bench.py --only gather_binned --reps 50 --ablate 4194304 || exit 1
done
tools/gpu_step.sh 300 $out/rocprof_split.log rocprofv3 --kernel-trace --stats -d $out/prof_split -o run -- python tools/gather_bench.py --only gather_binned --reps 24 || exit 1
echo done > $out/done
