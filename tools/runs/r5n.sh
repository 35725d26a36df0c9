set -o pipefail
# round 5 (n): the claim-space fragment copy with four chunks in flight per lane (asm
# loads, one wait) -- fragment parity, then A/B of cfg5 reassembly against the previous
# library (build_ab/libenethip_r5d.so), interleaved 3x, shuffled and in order, and a trace
out=gpurun_out/r5n
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fragments.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2 3; do
  tools/gpu_step.sh 300 $out/frag_new_$rep.log python tools/frag_bench.py --reps 30 || exit 1
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_r5d.so tools/gpu_step.sh 300 $out/frag_old_$rep.log python tools/frag_bench.py --reps 30 || exit 1
done
tools/gpu_step.sh 300 $out/frag_new_inorder.log python tools/frag_bench.py --reps 30 --in-order || exit 1
ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_r5d.so tools/gpu_step.sh 300 $out/frag_old_inorder.log python tools/frag_bench.py --reps 30 --in-order || exit 1
tools/gpu_step.sh 300 $out/rocprof_frag.log rocprofv3 --kernel-trace --stats -d $out/prof_frag -o run --output-format csv -- python tools/frag_bench.py --reps 20 || exit 1
echo done > $out/done
