set -o pipefail
# round 3 (j): in-place edge masking (vring), split binned gather (small segments in the join,
# compacted records with a device-side count): GPU suite, cfg3 / cfg5 / cfg2 / verify benches
out=gpurun_out/r3j
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/gather_p0_l8.log python -u tools/gather_bench.py --only gather_binned || exit 1
tools/gpu_step.sh 300 $out/gather_p0_l4.log python -u tools/gather_bench.py --only gather_binned --lanes 4 || exit 1
tools/gpu_step.sh 300 $out/gather_p13.log python -u tools/gather_bench.py --only gather_binned --path 13 || exit 1
tools/gpu_step.sh 300 $out/cfg3b_p0.json $B --config cfg3 --binned || exit 1
for l in 4 8; do for w in 1 2; do
  tools/gpu_step.sh 300 $out/cfg3b_p17_l${l}_w${w}.json $B --config cfg3 --binned --path 17 --lanes $l --wgs $w || exit 1
done; done
tools/gpu_step.sh 300 $out/cfg3_p0_l4.json $B --config cfg3 --lanes 4 || exit 1
tools/gpu_step.sh 300 $out/cfg3_p0.json $B --config cfg3 || exit 1
tools/gpu_step.sh 300 $out/cfg2_p0.json $B || exit 1
tools/gpu_step.sh 300 $out/verify_l20.log python -u tools/verify_bench.py --list 20 || exit 1
