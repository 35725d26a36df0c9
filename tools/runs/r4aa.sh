set -o pipefail
# round 4 (aa): single-batch launches by lanes per packet and workgroups per CU
out=gpurun_out/r4aa
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline --sustain-ms 0 --list 0 --streams 1"
for rep in 1 2; do
  for l in 4 8; do
    for w in 1 2; do
      tools/gpu_step.sh 200 $out/single_l${l}_w${w}_$rep.json $B --lanes $l --wgs $w || exit 1
    done
  done
  for l in 4 8; do
    tools/gpu_step.sh 300 $out/verify_l${l}_$rep.log python3 -u tools/verify_bench.py --reps 50 --list 5 --lanes $l || exit 1
  done
done
echo done > $out/done
