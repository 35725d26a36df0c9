set -o pipefail
# round 4 (m): dynamic rounds in the vring kernel -- GPU parity first (the whole
# -m gpu suite runs on them: they are the default), then the A/B against the static
# deal (diagnostics ablation 524288) serial and overlapped, cfg2 / cfg3 / cfg3 binned.
out=gpurun_out/r4m
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 240 $out/pytest_dyn.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "dynamic or cfg2 or binned" || exit 1
grep -q " passed" $out/pytest_dyn.log && ! grep -q "failed\|error" $out/pytest_dyn.log || { echo "parity failed"; exit 1; }
B="python bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for cfg in cfg2 cfg3; do
  for s in 1 6; do
    tools/gpu_step.sh 200 $out/${cfg}_s${s}_dyn.json $B --config $cfg --streams $s || exit 1
    tools/gpu_step.sh 200 $out/${cfg}_s${s}_static.json $B --config $cfg --streams $s --ablate 524288 || exit 1
  done
done
tools/gpu_step.sh 200 $out/cfg3b_dyn.json $B --config cfg3 --binned || exit 1
tools/gpu_step.sh 200 $out/cfg3b_static.json $B --config cfg3 --binned --ablate 524288 || exit 1
tools/gpu_step.sh 200 $out/timeline_l5_w2.log python -u tools/list_timeline.py 5 2 || exit 1
tools/gpu_step.sh 200 $out/timeline_l1_w1.log python -u tools/list_timeline.py 1 1 || exit 1
tools/gpu_step.sh 600 $out/pytest_all.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu || exit 1
echo done > $out/done
