set -o pipefail
# round 2: bench lines (driver form and default) + rocprof evidence for the vring kernel
out=gpurun_out/r2h
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
bash tools/profile_round.sh $out/prof || exit 1
