set -o pipefail
# round 6 (r): fragment reassembly -- the call against a plain device-to-device copy of the
# same bytes, and the per-kernel split under rocprof
out=gpurun_out/r6r
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 240 $out/frag.log python -u tools/frag_bench.py --reps 20 --copy-ref || exit 1
tools/gpu_step.sh 240 $out/frag_inorder.log python -u tools/frag_bench.py --reps 20 --in-order || exit 1
tools/gpu_step.sh 300 $out/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o frag -- python3 tools/frag_bench.py --reps 10 --copy-ref || exit 1
touch $out/done
