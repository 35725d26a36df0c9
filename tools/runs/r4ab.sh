set -o pipefail
# round 4 (ab): the driver form's value by batches per launch and streams
out=gpurun_out/r4ab
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for rep in 1 2; do
  for l in 1 2 5; do
    for s in 4 8 12; do
      tools/gpu_step.sh 200 $out/l${l}_s${s}_$rep.json $B --list $l --streams $s || exit 1
    done
  done
  tools/gpu_step.sh 200 $out/l5_s6_$rep.json $B || exit 1
done
echo done > $out/done
