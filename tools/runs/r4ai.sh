set -o pipefail
# round 4 (ai): the compact records instance (two workgroups per CU) -- binned parity tests,
# then A/B against one workgroup per CU: cfg3 binned (serial and 6-stream), its skeleton,
# the binned size scan, the cfg5 gather
out=gpurun_out/r4ai
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread -k "binned or gather" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --config cfg3 --binned"
for rep in 1 2; do
  for w in 1 2; do
    tools/gpu_step.sh 300 $out/cfg3b_w${w}_$rep.json $B --wgs $w || exit 1
    tools/gpu_step.sh 300 $out/cfg3b_s1_w${w}_$rep.json $B --wgs $w --streams 1 || exit 1
    tools/gpu_step.sh 300 $out/cfg3b_skel_s1_w${w}_$rep.json $B --wgs $w --streams 1 --ablate 38912 || exit 1
    tools/gpu_step.sh 300 $out/gather_w${w}_$rep.log python3 -u tools/gather_bench.py --only gather_binned --wgs $w || exit 1
  done
done
echo done > $out/done
