set -o pipefail
# round 2: driver-form comparison at equal work -- per-batch launches vs batch-list launches
out=gpurun_out/r2y
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  tools/gpu_step.sh 300 $out/d_single_$r.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/d_list5_$r.json python bench.py --steps 4 --warmup 2 --list 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/d_list5_s2_$r.json python bench.py --steps 4 --warmup 2 --list 5 --streams 2 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/d_list2_$r.json python bench.py --steps 10 --warmup 2 --list 2 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/d_list5_w2_$r.json python bench.py --steps 4 --warmup 2 --list 5 --wgs 2 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/l_single_$r.json python bench.py --steps 200 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/l_list5_$r.json python bench.py --steps 40 --list 5 --no-cpu-baseline || exit 1
done
