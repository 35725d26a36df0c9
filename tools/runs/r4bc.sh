set -o pipefail
# round 4 (bc): fragment reassembly with the fragments in send order against shuffled (the
# decide kernel's descriptor stores then land in command order), kernel traces of both
out=gpurun_out/r4bc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_shuffled -o run --output-format csv -- python3 tools/frag_bench.py > $out/frag_shuffled.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_inorder -o run --output-format csv -- python3 tools/frag_bench.py --in-order > $out/frag_inorder.log 2>&1 || exit 1
echo done > $out/done
