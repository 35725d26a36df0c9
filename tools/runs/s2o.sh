set -o pipefail
# round 2 (session 3): driver-form bench (--steps 20 --warmup 5): graph replay vs direct launches, list/stream variants
out=gpurun_out/s2o
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  tools/gpu_step.sh 200 $out/graph_$i.json python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/direct_$i.json python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --launch direct || exit 1
done
tools/gpu_step.sh 200 $out/list10_s2.json python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --list 10 --rotate 10 --streams 2 || exit 1
tools/gpu_step.sh 200 $out/list20.json python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --list 20 --rotate 20 --streams 1 || exit 1
tools/gpu_step.sh 200 $out/list4_s5.json python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --list 4 --streams 5 || exit 1
tools/gpu_step.sh 200 $out/list2_s10.json python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --list 2 --streams 10 || exit 1
