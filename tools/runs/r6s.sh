set -o pipefail
# round 6 (s): fragment copy in arena order (the atomic path's frag_copy_kernel, forced by a
# large bitmap: --words 64) against the claim-order copy, per kernel under rocprof
out=gpurun_out/r6s
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 240 $out/frag_w64.log python -u tools/frag_bench.py --reps 20 --words 64 || exit 1
tools/gpu_step.sh 300 $out/prof_w64.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_w64 -o frag -- python3 tools/frag_bench.py --reps 10 --words 64 || exit 1
tools/gpu_step.sh 300 $out/prof_w2.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_w2 -o frag -- python3 tools/frag_bench.py --reps 10 --copy-ref || exit 1
touch $out/done
