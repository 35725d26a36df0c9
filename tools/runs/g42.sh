set -o pipefail
out=gpurun_out/g42
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fragments.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_frag.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/frag_bench.py > $out/frag.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/frag_trace -o run --output-format csv -- python3 tools/frag_bench.py --reps 10 > $out/frag_rocprof.log 2>&1 || exit 1
