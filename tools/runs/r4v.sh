set -o pipefail
# round 4 (v): pair rounds (diagnostics ablation 8388608) against the static deal
out=gpurun_out/r4v
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_sel.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "dynamic" || exit 1
grep -q " passed" $out/pytest_sel.log && ! grep -q " failed" $out/pytest_sel.log || { echo "parity failed"; exit 1; }
B="python bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for rep in 1 2; do
  for cfg in "--streams 1" "--config cfg3 --streams 1" "--config cfg3 --binned --streams 1" "--list 20 --rotate 20 --streams 1"; do
    tag=$(echo "x$cfg" | tr -d ' -' )
    tools/gpu_step.sh 200 $out/static_${tag}_$rep.json $B $cfg || exit 1
    tools/gpu_step.sh 200 $out/pair_${tag}_$rep.json $B $cfg --ablate 8388608 || exit 1
  done
done
echo done > $out/done
