#!/bin/bash
# Instruction-mix and stall counters for one configuration, one --pmc group per
# run (never combined with trace domains).  Usage:
#   tools/pmc_mix.sh OUTDIR args-for-profile_one...
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -e
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 tools/profile_one.py "$@"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM -d "$out/mix" -o run --output-format csv -- python3 tools/profile_one.py "$@"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d "$out/sq" -o run --output-format csv -- python3 tools/profile_one.py "$@"
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$out/lds" -o run --output-format csv -- python3 tools/profile_one.py "$@"
