set -o pipefail
# round 2 (session 3): binned records on the vring kernel -- parity, cfg3 bench (vring vs lean records), rocprof
out=gpurun_out/s2q
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest_binned.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "binned" || exit 1
grep -q " passed" $out/pytest_binned.log || exit 1
grep -q "FAILED\|Timeout" $out/pytest_binned.log && exit 1
tools/gpu_step.sh 300 $out/cfg3_vring_binned.json python bench.py --config cfg3 --binned --lanes 4 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/cfg3_vring_binned_l8.json python bench.py --config cfg3 --binned --lanes 8 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/cfg3_lean_binned.json python bench.py --config cfg3 --binned --lanes 4 --path 13 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/cfg3_vring_list.json python bench.py --config cfg3 --lanes 4 --no-cpu-baseline || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --config cfg3 --binned --lanes 4 --streams 1 --steps 50 --warmup 5 --no-cpu-baseline > $out/cfg3_rocprof.json 2>&1 || exit 1
