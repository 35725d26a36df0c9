#!/bin/bash
# Counter passes for one configuration (each --pmc group in its own run, no
# trace domains combined with --pmc).  Usage: tools/pmc_run.sh OUTDIR args-for-profile_one...
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -e
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 tools/profile_one.py "$@"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python3 tools/profile_one.py "$@"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d "$out/sq" -o run --output-format csv -- python3 tools/profile_one.py "$@"
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d "$out/lds" -o run --output-format csv -- python3 tools/profile_one.py "$@"
