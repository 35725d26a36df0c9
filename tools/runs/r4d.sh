set -o pipefail
# round 4 (d): where a serial launch loses against overlapped ones (per-wave end
# times of 1-, 5- and 20-batch launches), and the sustained-rate cause (VERDICT r3
# #6): the product, its no-lookup ablation and its skeleton beside the read probe,
# with the amdsmi refresh logged.
out=gpurun_out/r4d
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/timeline_l5_w2.log python -u tools/list_timeline.py 5 2 || exit 1
tools/gpu_step.sh 200 $out/timeline_l20_w2.log python -u tools/list_timeline.py 20 2 || exit 1
tools/gpu_step.sh 200 $out/timeline_l1_w1.log python -u tools/list_timeline.py 1 1 || exit 1
tools/gpu_step.sh 300 $out/sustain_vring.log python -u tools/sustain.py --kernel vring --launches 3000 || exit 1
tools/gpu_step.sh 300 $out/sustain_abl4096.log python -u tools/sustain.py --kernel vring --launches 3000 --ablate 4096 || exit 1
tools/gpu_step.sh 300 $out/sustain_skel.log python -u tools/sustain.py --kernel vring --launches 3000 --ablate 38912 || exit 1
tools/gpu_step.sh 300 $out/sustain_probe.log python -u tools/sustain.py --kernel probe --launches 3000 || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 200 $out/bench_s2.json $B --streams 2 || exit 1
tools/gpu_step.sh 200 $out/bench_s4.json $B --streams 4 || exit 1
echo done > $out/done
