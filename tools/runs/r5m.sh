set -o pipefail
# round 5 (m): with the cheaper fold, do the traffic-saving tail-first order (path 21)
# or nontemporal stage loads (18) now pay on cfg2?  Interleaved 3x, driver form
out=gpurun_out/r5m
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for p in 0 21 18; do
    tools/gpu_step.sh 300 $out/bench_p${p}_$rep.json python bench.py --path $p --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  done
done
echo done > $out/done
