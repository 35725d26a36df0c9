set -o pipefail
# round 5 (af): fragment copy with nontemporal 16-byte loads and stores (libenethip_fragnt)
# against the product (r5f): the fragment GPU tests on the nt library, then
# tools/frag_bench.py interleaved 3x (cfg5 shuffled), and in order once each
out=gpurun_out/r5af
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_fragnt.so tools/gpu_step.sh 600 $out/pytest_frag_nt.log python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fragments.py || exit 1
grep -q " passed" $out/pytest_frag_nt.log || exit 1
grep -q "FAILED" $out/pytest_frag_nt.log && exit 1
for rep in 1 2 3; do
  for v in r5f fragnt; do
    ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so tools/gpu_step.sh 300 $out/frag_${v}_$rep.log python tools/frag_bench.py --reps 30 || exit 1
  done
done
for v in r5f fragnt; do
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so tools/gpu_step.sh 300 $out/frag_${v}_inorder.log python tools/frag_bench.py --reps 30 --in-order || exit 1
done
echo done > $out/done
