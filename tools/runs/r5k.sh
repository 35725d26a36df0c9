set -o pipefail
# round 5 (k): the split gather join, tuned (78 VGPRs so every block is resident; two
# segments per post-join thread) -- gather parity, then A/B against the one-pass join
# in the diagnostics build (4194304), interleaved 3x, and a kernel trace
out=gpurun_out/r5k
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread -k "gather" tests/test_gpu_parity.py tests/test_gpu_harness.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2 3; do
  tools/gpu_step.sh 300 $out/split_$rep.log python tools/gather_bench.py --only gather_binned --reps 50 || exit 1
  tools/gpu_step.sh 300 $out/onepass_$rep.log python tools/gather_bench.py --only gather_binned --reps 50 --ablate 4194304 || exit 1
done
tools/gpu_step.sh 300 $out/rocprof_split.log rocprofv3 --kernel-trace --stats -d $out/prof_split -o run --output-format csv -- python tools/gather_bench.py --only gather_binned --reps 24 || exit 1
tools/gpu_step.sh 300 $out/rocprof_onepass.log rocprofv3 --kernel-trace --stats -d $out/prof_onepass -o run --output-format csv -- python tools/gather_bench.py --only gather_binned --reps 24 --ablate 4194304 || exit 1
echo done > $out/done
