set -o pipefail
# round 2: vring with metadata by LDS-DMA, metadata once per group, ring in v48-v63, asm shuffle
out=gpurun_out/r2v
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/listprobe.log python -u tools/listprobe.py || exit 1
grep -q "^done" $out/listprobe.log || exit 1
tools/gpu_step.sh 300 $out/pytest_new.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "empty or vring or batch_list or cfg2 or golden or random or cfg3" || exit 1
grep -q " passed" $out/pytest_new.log || exit 1
grep -q "failed\|Timeout" $out/pytest_new.log && exit 1
for w in 1 2; do
  tools/gpu_step.sh 300 $out/bench_w${w}.json python bench.py --wgs $w --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/bench_list5_w${w}.json python bench.py --list 5 --wgs $w --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/bench_list5_w${w}_s1.json python bench.py --list 5 --wgs $w --streams 1 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/bench_l8_w${w}.json python bench.py --lanes 8 --wgs $w --no-cpu-baseline || exit 1
done
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d $out/p1_w2 -o run --output-format csv -- python3 tools/profile_one.py --reps 20 --lanes 4 --list 5 --wgs 2 > $out/p1_w2.log 2>&1 || echo "p1 failed"
