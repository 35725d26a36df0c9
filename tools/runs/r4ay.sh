set -o pipefail
# round 4 (ay): range coder input read 16 bytes at a time against one byte at a time
# (the previous library), interleaved; the GPU range coder parity tests on the new one
out=gpurun_out/r4ay
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests/test_gpu_range_coder.py -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2 3; do
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_base.so tools/gpu_step.sh 300 $out/rc_base_$rep.log python3 -u tools/rc_bench.py || exit 1
  ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_win.so tools/gpu_step.sh 300 $out/rc_win_$rep.log python3 -u tools/rc_bench.py || exit 1
done
echo done > $out/done
