set -o pipefail
# round 4 (bd): fragment reassembly with slot-major (claim-space) copy descriptors --
# the fragment GPU parity tests first, then frag_bench shuffled / in order with traces
out=gpurun_out/r4bd
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "frag" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_shuffled -o run --output-format csv -- python3 tools/frag_bench.py > $out/frag_shuffled.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_inorder -o run --output-format csv -- python3 tools/frag_bench.py --in-order > $out/frag_inorder.log 2>&1 || exit 1
tools/gpu_step.sh 300 $out/frag_2.log python3 -u tools/frag_bench.py || exit 1
echo done > $out/done
