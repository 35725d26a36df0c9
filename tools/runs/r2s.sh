set -o pipefail
# round 2: vring at 2 workgroups per CU in one launch (more bytes in flight), single and list
out=gpurun_out/r2s
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_new.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "vring or batch_list or cfg2" || exit 1
for w in 1 2; do
  tools/gpu_step.sh 300 $out/bench_w${w}.json python bench.py --wgs $w --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/bench_w${w}_s1.json python bench.py --wgs $w --streams 1 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/bench_list5_w${w}.json python bench.py --list 5 --wgs $w --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/bench_list5_w${w}_s1.json python bench.py --list 5 --wgs $w --streams 1 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/bench_l8_w${w}.json python bench.py --lanes 8 --wgs $w --no-cpu-baseline || exit 1
done
