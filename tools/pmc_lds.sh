#!/bin/bash
# LDS bank-conflict counters for several "path:lanes:ablate" configurations.
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -e
for cfg in "$@"; do
  IFS=: read p l a <<< "$cfg"
  timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d "$out/p${p}_l${l}_a${a}" -o run --output-format csv -- python3 tools/profile_one.py --path $p --lanes $l --ablate $a --reps 3 > "$out.p${p}_l${l}_a${a}.log" 2>&1
  echo "== $cfg"; python3 tools/pmc_summary.py "$out/p${p}_l${l}_a${a}" crc32
done
