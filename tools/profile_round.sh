#!/bin/bash
# Round evidence for profiles/ (run on the GPU box): tools/profile_round.sh OUTDIR
#  1. rocprofv3 --kernel-trace --stats of the default bench command (4 streams:
#     overlapping launches, so per-kernel durations there include sharing the GPU);
#  2. the same with --streams 1: every launch alone, the kernel's own duration;
#  3. a separate --pmc FETCH_SIZE pass (HBM bytes per launch).
out=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -e
mkdir -p "$out"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/bench_trace" -o run --output-format csv \
    -- python3 bench.py --steps 50 --warmup 10 --cpu-seconds 2 > "$out/bench_under_rocprof.json" 2> "$out/bench_under_rocprof.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/bench_s1_trace" -o run --output-format csv \
    -- python3 bench.py --steps 50 --warmup 10 --streams 1 --no-cpu-baseline > "$out/bench_s1_under_rocprof.json" 2> "$out/bench_s1_under_rocprof.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv \
    -- python3 tools/profile_one.py --reps 20 --probe --list 5 --wgs 2 > "$out/fetch.log" 2>&1
python3 tools/traffic.py "$out/fetch" 78643200 5 "$out/traffic_cfg2.json"
