set -o pipefail
# round 5 (ag): the gather join's first segFirst pair loaded before its table fill --
# binned gather GPU tests on the new library, gather_bench interleaved 3x against r5f,
# then the kernel trace of both (join kernel mean)
out=gpurun_out/r5ag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_join.so tools/gpu_step.sh 600 $out/pytest_gather.log python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "gather" || exit 1
grep -q " passed" $out/pytest_gather.log || exit 1
grep -q "FAILED" $out/pytest_gather.log && exit 1
for rep in 1 2 3; do
  for v in r5f join; do
    ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so tools/gpu_step.sh 300 $out/gather_${v}_$rep.log python -u tools/gather_bench.py --only gather_binned --reps 50 || exit 1
  done
done
for v in r5f join; do
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$v -o run --output-format csv -- python3 tools/gather_bench.py --only gather_binned --reps 24 > $out/prof_$v.log 2>&1 || exit 1
done
echo done > $out/done
