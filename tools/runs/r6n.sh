set -o pipefail
# round 6 (n): local tiles at two packets per thread, also for the binned gather's
# segment pass: the GPU suite, smoke, cfg3 binned and cfg5 gather A/B against path 17
out=gpurun_out/r6n
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 900 $out/pytest_gpu.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu || exit 1
tools/gpu_step.sh 200 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2; do
  tools/gpu_step.sh 300 $out/gather_local_$rep.log python -u tools/gather_bench.py --only gather_binned
  tools/gpu_step.sh 300 $out/gather_two_$rep.log python -u tools/gather_bench.py --only gather_binned --path 17
  tools/gpu_step.sh 300 $out/cfg3b_ser_$rep.json $B --config cfg3 --binned --streams 1 --sustain-ms 0
  tools/gpu_step.sh 300 $out/cfg3b_two_ser_$rep.json $B --config cfg3 --binned --streams 1 --sustain-ms 0 --path 17 --wgs 2
  tools/gpu_step.sh 300 $out/cfg3b_drv_$rep.json $B --config cfg3 --binned
done
touch $out/done
