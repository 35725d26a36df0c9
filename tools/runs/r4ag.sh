set -o pipefail
# round 4 (ag): the binned entry's serial rate against batch size (plain and skeleton)
out=gpurun_out/r4ag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/binned_plain.log python3 -u tools/binned_bench.py || exit 1
tools/gpu_step.sh 300 $out/binned_skel.log python3 -u tools/binned_bench.py --ablate 38912 || exit 1
tools/gpu_step.sh 120 $out/alignprobe_1m.txt ./tools/alignprobe_bin 1000000 || exit 1
tools/gpu_step.sh 120 $out/alignprobe_512k.txt ./tools/alignprobe_bin 524288 || exit 1
echo done > $out/done
