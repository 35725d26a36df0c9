set -o pipefail
# round 3 (t): EA windows only for 16-byte-aligned packet ends (aligned loads); binned + gather tests, cfg3 / cfg5 timings
out=gpurun_out/r3t
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py -m gpu -v --timeout 240 --timeout-method thread -k "gather or binned or bin or verify" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for r in 1 2; do
  tools/gpu_step.sh 300 $out/gather_$r.log python -u tools/gather_bench.py --only gather_binned || exit 1
done
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/cfg3b_1.json $B --config cfg3 --binned || exit 1
tools/gpu_step.sh 300 $out/cfg3b_2.json $B --config cfg3 --binned || exit 1
