set -o pipefail
out=gpurun_out/g21
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/bench_s1_trace -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --streams 1 --no-cpu-baseline > $out/bench_s1_under_rocprof.json 2> $out/bench_s1_under_rocprof.err || exit 1
tools/gpu_step.sh 300 $out/bench_cfg3.json python bench.py --config cfg3 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_cfg3_l4.json python bench.py --config cfg3 --lanes 4 --no-cpu-baseline || exit 1
