set -o pipefail
# round 2: where does the vring kernel's time go -- SQ counters, single launches vs batch list
out=gpurun_out/r2t
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
i=0
for args in "--lanes 4" "--lanes 4 --list 5" "--lanes 8" "--lanes 4 --probe"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P1 -d $out/p1_$i -o run --output-format csv -- python3 tools/profile_one.py --reps 20 $args > $out/p1_$i.log 2>&1 || { echo "p1 $i failed"; tail -5 $out/p1_$i.log; }
  timeout -s KILL 90 rocprofv3 --pmc $P2 -d $out/p2_$i -o run --output-format csv -- python3 tools/profile_one.py --reps 20 $args > $out/p2_$i.log 2>&1 || { echo "p2 $i failed"; tail -5 $out/p2_$i.log; }
done
