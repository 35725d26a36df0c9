set -o pipefail
# round 6 (m): the one-launch binned default (local tiles, two workgroups per CU): the GPU
# suite, smoke, cfg3 binned (serial and driver form, x2) and the cfg2 default line
out=gpurun_out/r6m
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 900 $out/pytest_gpu.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu
tools/gpu_step.sh 200 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2; do
  tools/gpu_step.sh 300 $out/cfg3b_ser_$rep.json $B --config cfg3 --binned --streams 1 --sustain-ms 0
  tools/gpu_step.sh 300 $out/cfg3b_drv_$rep.json $B --config cfg3 --binned
  tools/gpu_step.sh 300 $out/cfg3b_two_drv_$rep.json $B --config cfg3 --binned --path 17 --wgs 2
done
tools/gpu_step.sh 300 $out/cfg2_drv.json $B
touch $out/done
