set -o pipefail
# round 2: rocprof evidence for the vring kernel (default bench, serial bench, FETCH_SIZE)
# and cfg3 (mixed lengths): vring unbinned vs lean binned
out=gpurun_out/r2o
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh $out/prof || exit 1
tools/gpu_step.sh 300 $out/cfg3_vring_l4.json python bench.py --config cfg3 --no-cpu-baseline --steps 100 || exit 1
tools/gpu_step.sh 300 $out/cfg3_vring_l8.json python bench.py --config cfg3 --lanes 8 --no-cpu-baseline --steps 100 || exit 1
tools/gpu_step.sh 300 $out/cfg3_binned_l4.json python bench.py --config cfg3 --binned --no-cpu-baseline --steps 100 || exit 1
