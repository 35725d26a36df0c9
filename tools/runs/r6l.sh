set -o pipefail
# round 6 (l): the one-launch binned checksum, first two groups' metadata in LDS from the sort:
# timelines (local at one and two workgroups per CU, two-launch at two) and the A/B
out=gpurun_out/r6l
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_binned.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "binned or local"
tools/gpu_step.sh 200 $out/timeline_local_w1.log python tools/bin_timeline.py 3 1 0
tools/gpu_step.sh 200 $out/timeline_two_w1.log python tools/bin_timeline.py 3 1 17

B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --config cfg3 --binned"
for rep in 1 2; do
  for w in 1 2; do
    tools/gpu_step.sh 300 $out/local_w${w}_$rep.json $B --wgs $w --streams 1 --sustain-ms 0
  done
  tools/gpu_step.sh 300 $out/two_w2_$rep.json $B --wgs 2 --streams 1 --sustain-ms 0 --path 17
done
touch $out/done
