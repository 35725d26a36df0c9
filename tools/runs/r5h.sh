set -o pipefail
# round 5 (h): vring VALU cut (in-place fused fold, interior-stage addresses, integer
# 64-bit min/max): the GPU suite on the new library, then A/B against the round-4 HEAD
# library (build_ab/libenethip_base.so), interleaved 3x on one box
out=gpurun_out/r5h
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 900 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2 3; do
  for v in base r5a; do
    ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so tools/gpu_step.sh 300 $out/bench_${v}_$rep.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so tools/gpu_step.sh 300 $out/cfg3b_${v}_$rep.json python bench.py --config cfg3 --binned --steps 20 --warmup 5 --no-cpu-baseline || exit 1
    ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so tools/gpu_step.sh 300 $out/verify_${v}_$rep.log python tools/verify_bench.py --list 20 || exit 1
    ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so tools/gpu_step.sh 300 $out/gather_${v}_$rep.log python tools/gather_bench.py || exit 1
  done
done
echo done > $out/done
