set -o pipefail
# round 4 (af): cfg3 binned in the serial form (one stream): plain, no-lookup and skeleton
# ablations, bench lines and a kernel trace each
out=gpurun_out/r4af
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --config cfg3 --binned --streams 1"
for rep in 1 2; do
  for a in 0 4096 38912; do
    tools/gpu_step.sh 300 $out/cfg3b_s1_a${a}_$rep.json $B --ablate $a || exit 1
  done
done
for a in 0 38912; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_a$a -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 --config cfg3 --binned --streams 1 --ablate $a > $out/prof_a$a.log 2>&1 || exit 1
done
echo done > $out/done
