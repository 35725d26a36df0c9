set -o pipefail
# round 2 (session 4): cfg4 (1 M x 1200 B, one shard at N=1: strong-scaling config) and cfg3 at HEAD
out=gpurun_out/s3i
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/cfg4_driver.json python bench.py --config cfg4 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/cfg4_l1.json python bench.py --config cfg4 --steps 20 --warmup 5 --list 1 --streams 1 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/cfg3_binned.json python bench.py --config cfg3 --binned --lanes 4 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/cfg3_list.json python bench.py --config cfg3 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
