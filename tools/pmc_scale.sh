#!/bin/bash
# VALU/LDS/SALU instruction counts and kernel time vs packet size at ~equal bytes:
# separates per-byte from per-packet cost.  tools/pmc_scale.sh OUTDIR lanes cfg...
out=$1; lanes=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -e
for cfg in "$@"; do
  d="$out/$(echo $cfg | tr ':' '_')_l$lanes"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$d/trace" -o run --output-format csv -- python3 tools/profile_one.py --config $cfg --lanes $lanes --reps 10 --rotate 3 > /dev/null 2>&1
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d "$d/mix" -o run --output-format csv -- python3 tools/profile_one.py --config $cfg --lanes $lanes --reps 3 --rotate 3 > /dev/null 2>&1
  echo "== $cfg lanes=$lanes"; python3 tools/pmc_summary.py "$d/mix" crc32
  grep crc32 "$d/trace/run_kernel_stats.csv" | cut -d, -f2-4
done
