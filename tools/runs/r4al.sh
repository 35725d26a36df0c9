set -o pipefail
# round 4 (al): the binned gather at two workgroups per CU by default (compact records
# instance) -- gather / binned parity, then default against --wgs 1, interleaved, and a
# kernel trace of the default
out=gpurun_out/r4al
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread -k "binned or gather" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2 3; do
  for w in 0 1; do
    tools/gpu_step.sh 300 $out/gather_w${w}_$rep.log python3 -u tools/gather_bench.py --only gather_binned --wgs $w || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/gather_trace -o run --output-format csv -- python3 tools/gather_bench.py --only gather_binned > $out/gather_trace.log 2>&1 || exit 1
echo done > $out/done
