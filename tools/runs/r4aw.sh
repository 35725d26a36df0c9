set -o pipefail
# round 4 (aw): fragment claim kernel with a plain store in place of its atomicMin (a probe
# library; cfg5 has no duplicate fragments, so results stay exact) against the product,
# interleaved, with kernel traces
out=gpurun_out/r4aw
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base noatomic; do
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$v -o run --output-format csv -- python3 tools/frag_bench.py > $out/frag_$v.log 2>&1 || exit 1
done
echo done > $out/done
