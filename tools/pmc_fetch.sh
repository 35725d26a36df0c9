#!/bin/bash
# FETCH_SIZE for several (path, lanes) configurations: tools/pmc_fetch.sh OUTDIR "path:lanes" ...
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -e
timeout -k 10 120 rocprofv3 -L > "$out.counters.txt" 2>&1 || true
for cfg in "$@"; do
  p=${cfg%%:*}; l=${cfg##*:}
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$out/p${p}_l${l}" -o run --output-format csv -- python3 tools/profile_one.py --path $p --lanes $l --reps 10
done
