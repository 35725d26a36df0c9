set -o pipefail
# round 6 (t): the atomic decide path's overlap check (frag_clash_kernel): fragment tests,
# cfg5 on both decide paths (words 2 = slots, words 64 = atomic), per-kernel split
out=gpurun_out/r6t
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest_frag.log python -u -m pytest tests/test_gpu_fragments.py tests/test_fragments.py -x -v --timeout 120 --timeout-method thread || exit 1
tools/gpu_step.sh 240 $out/frag_w2.log python -u tools/frag_bench.py --reps 20 || exit 1
tools/gpu_step.sh 240 $out/frag_w64.log python -u tools/frag_bench.py --reps 20 --words 64 || exit 1
tools/gpu_step.sh 300 $out/prof_w64.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_w64 -o frag -- python3 tools/frag_bench.py --reps 10 --words 64 || exit 1
touch $out/done
