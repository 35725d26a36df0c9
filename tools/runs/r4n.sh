set -o pipefail
# round 4 (n): why the dynamic rounds ran 2x slower (end records of both deals), and
# what bounds the gather join (ablations under a kernel trace)
out=gpurun_out/r4n
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/pytest_join.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "segment_parallel or dynamic or gather_binned" || exit 1
tools/gpu_step.sh 200 $out/dyn_probe_l5_w2.log python -u tools/dyn_probe.py 5 2 8 || exit 1
tools/gpu_step.sh 200 $out/dyn_probe_l1_w1.log python -u tools/dyn_probe.py 1 1 8 || exit 1
for j in 0 1 2 3 5 7 8; do
  tools/gpu_step.sh 200 $out/gather_j$j.log rocprofv3 --kernel-trace --stats -d $out/prof_j$j -o run -- python3 -u tools/gather_bench.py --only gather_binned --reps 20 --ablate $((j * 1048576)) || exit 1
done
tools/gpu_step.sh 200 $out/gather_dyn.log python3 -u tools/gather_bench.py --only gather_binned --reps 20 --ablate 524288 || exit 1
tools/gpu_step.sh 300 $out/gather_cpu.log python3 -u tools/gather_bench.py --only gather_binned --reps 20 --cpu-seconds 20 || exit 1
echo done > $out/done
