set -o pipefail
# round 3 (4j): the driver-form bench at 4 / 5 / 10 / 20 batches per launch (same 20 steps), interleaved
out=gpurun_out/r4j
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for r in 1 2; do
  for l in 4 5 10 20; do
    tools/gpu_step.sh 300 $out/list${l}_$r.json $B --list $l || exit 1
  done
done
