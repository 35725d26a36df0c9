set -o pipefail
# round 2: per-wave timelines (vring l4 / l8, lean l8) and the lean kernel's serial bench for reference
out=gpurun_out/r2x
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/tl_vring_l4.log python -u tools/timeline.py --lanes 4 --path 0 || exit 1
tools/gpu_step.sh 200 $out/tl_vring_l8.log python -u tools/timeline.py --lanes 8 --path 0 || exit 1
tools/gpu_step.sh 200 $out/tl_lean_l8.log python -u tools/timeline.py --lanes 8 --path 13 || exit 1
tools/gpu_step.sh 300 $out/bench_lean_l8_s1.json python bench.py --lanes 8 --path 13 --streams 1 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_lean_l8.json python bench.py --lanes 8 --path 13 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
