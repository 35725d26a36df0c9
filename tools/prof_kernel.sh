#!/bin/bash
# Per-kernel evidence for one configuration (run on the GPU box):
#   tools/prof_kernel.sh OUTDIR NAME BATCHES_PER_LAUNCH [profile_one.py args ...]
#  1. rocprofv3 --kernel-trace --stats over 100 serial launches (the kernel's own duration);
#  2. a separate --pmc FETCH_SIZE pass (+ the read probe as calibration) -> traffic JSON.
out=$1; name=$2; per=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -e
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/${name}_trace" -o run --output-format csv \
    -- python3 tools/profile_one.py --reps $((100 * per)) --list $per "$@" > "$out/${name}_trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$out/${name}_fetch" -o run --output-format csv \
    -- python3 tools/profile_one.py --reps $((4 * per)) --list $per --probe "$@" > "$out/${name}_fetch.log" 2>&1
python3 tools/traffic.py "$out/${name}_fetch" 78643200 $per "$out/${name}_traffic.json" > /dev/null
