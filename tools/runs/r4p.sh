set -o pipefail
# round 4 (p): join with unconditional spread loads; dynamic rounds with the dead-claim skip
# claim word, no end-of-launch atomics, three static rounds) against the static deal
out=gpurun_out/r4p
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_sel.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_harness.py -k "dynamic or gather or cfg2 or binned or verify" || exit 1
grep -q " passed" $out/pytest_sel.log && ! grep -q " failed" $out/pytest_sel.log || { echo "parity failed"; exit 1; }
tools/gpu_step.sh 200 $out/gather_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_gather -o run -- python3 -u tools/gather_bench.py --only gather_binned --reps 20 || exit 1
tools/gpu_step.sh 200 $out/dyn_probe_l5_w2.log python -u tools/dyn_probe.py 5 2 8 || exit 1
B="python bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for rep in 1; do
  tools/gpu_step.sh 200 $out/cfg2_s1_static_$rep.json $B --streams 1 || exit 1
  tools/gpu_step.sh 200 $out/cfg2_s1_dyn_$rep.json $B --streams 1 --ablate 524288 || exit 1
  tools/gpu_step.sh 200 $out/cfg2_s6_static_$rep.json $B || exit 1
  tools/gpu_step.sh 200 $out/cfg2_s6_dyn_$rep.json $B --ablate 524288 || exit 1
done
tools/gpu_step.sh 200 $out/cfg2_l0_static.json $B --list 0 --streams 1 || exit 1
tools/gpu_step.sh 200 $out/cfg2_l0_dyn.json $B --list 0 --streams 1 --ablate 524288 || exit 1
tools/gpu_step.sh 200 $out/cfg3b_static.json $B --config cfg3 --binned || exit 1
tools/gpu_step.sh 200 $out/cfg3b_dyn.json $B --config cfg3 --binned --ablate 524288 || exit 1
tools/gpu_step.sh 200 $out/cfg3_static.json $B --config cfg3 || exit 1
tools/gpu_step.sh 200 $out/cfg3_dyn.json $B --config cfg3 --ablate 524288 || exit 1
echo done > $out/done
