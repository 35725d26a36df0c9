set -o pipefail
# round 4 (ar): fragment copy with nt loads / stores against the previous library, interleaved
out=gpurun_out/r4ar
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_base.so tools/gpu_step.sh 300 $out/frag_base_$rep.log python3 -u tools/frag_bench.py || exit 1
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_nt.so tools/gpu_step.sh 300 $out/frag_nt_$rep.log python3 -u tools/frag_bench.py || exit 1
done
echo done > $out/done
