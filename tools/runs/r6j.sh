set -o pipefail
# round 6 (j): the one-launch binned checksum (local tiles, BIN = 3): binned GPU tests,
# then cfg3 binned A/B against the two-launch form (path 17), one and two workgroups per CU
out=gpurun_out/r6j
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest_binned.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "binned or local"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --config cfg3 --binned"
for rep in 1 2; do
  for w in 1 2; do
    tools/gpu_step.sh 300 $out/local_w${w}_$rep.json $B --wgs $w --streams 1 --sustain-ms 0
    tools/gpu_step.sh 300 $out/two_w${w}_$rep.json $B --wgs $w --streams 1 --sustain-ms 0 --path 17
  done
done
tools/gpu_step.sh 300 $out/local_default_drv.json $B
tools/gpu_step.sh 300 $out/two_default_drv.json $B --path 17
touch $out/done
