set -o pipefail
# round 4 (q): join A/B (round 3's against the batched-load join), dynamic rounds
# v2 + no claim when the static rounds cover the launch
out=gpurun_out/r4q
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_sel.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_harness.py -k "dynamic or gather or binned" || exit 1
grep -q " passed" $out/pytest_sel.log && ! grep -q " failed" $out/pytest_sel.log || { echo "parity failed"; exit 1; }
tools/gpu_step.sh 200 $out/gather_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_gather -o run -- python3 -u tools/gather_bench.py --only gather_binned --reps 20 || exit 1
tools/gpu_step.sh 200 $out/gather_prof_r3.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_gather_r3 -o run -- python3 -u tools/gather_bench.py --only gather_binned --reps 20 --ablate 8388608 || exit 1
B="python bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 200 $out/cfg2_s1_static.json $B --streams 1 || exit 1
tools/gpu_step.sh 200 $out/cfg2_s1_dyn.json $B --streams 1 --ablate 524288 || exit 1
tools/gpu_step.sh 200 $out/cfg2_l0_dyn.json $B --list 0 --streams 1 --ablate 524288 || exit 1
tools/gpu_step.sh 200 $out/cfg3_static.json $B --config cfg3 || exit 1
tools/gpu_step.sh 200 $out/cfg3_dyn.json $B --config cfg3 --ablate 524288 || exit 1
echo done > $out/done
