set -o pipefail
# round 4 (u): late next-group takes (the wave's next slot taken two stages before the end
# of its group, every slot after the first from the workgroup's counter) -- the whole
# -m gpu suite, then A/B against the previous build (ENET_HIP_LIBRARY=ab/libenethip_prev.so)
out=gpurun_out/r4u
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 900 $out/pytest_all.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu || exit 1
grep -q " passed" $out/pytest_all.log && ! grep -q " failed" $out/pytest_all.log || { echo "parity failed"; exit 1; }
PREV=enet-csharp_amd/ab/libenethip_prev.so
B="python bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for rep in 1 2; do
  for cfg in "" "--list 0 --streams 1" "--config cfg3" "--config cfg3 --binned"; do
    tag=$(echo "x$cfg" | tr -d ' -' )
    tools/gpu_step.sh 200 $out/new_${tag}_$rep.json $B --streams 1 $cfg || exit 1
    ENET_HIP_LIBRARY=$PREV tools/gpu_step.sh 200 $out/prev_${tag}_$rep.json $B --streams 1 $cfg || exit 1
  done
  tools/gpu_step.sh 200 $out/new_driver_$rep.json $B || exit 1
  ENET_HIP_LIBRARY=$PREV tools/gpu_step.sh 200 $out/prev_driver_$rep.json $B || exit 1
done
tools/gpu_step.sh 200 $out/timeline_l5_w2_p8.log python -u tools/list_timeline.py 5 2 8 || exit 1
tools/gpu_step.sh 200 $out/timeline_l1_w1_p8.log python -u tools/list_timeline.py 1 1 8 || exit 1
echo done > $out/done
