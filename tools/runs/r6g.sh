set -o pipefail
# round 6 (g): kernel traces of the PCIe probe (the same clock as the receive kernels' traces),
# and the single-batch cfg2 timeline
out=gpurun_out/r6g
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/probe_trace -o run --output-format csv -- ./tools/pcieprobe > $out/pcieprobe.log 2>&1 || exit 1
tools/gpu_step.sh 300 $out/timeline_single_w1.log python -u tools/list_timeline.py 1 1 8 || exit 1
tools/gpu_step.sh 300 $out/timeline_single_w2.log python -u tools/list_timeline.py 1 2 8 || exit 1
tools/gpu_step.sh 300 $out/timeline_list5_w2.log python -u tools/list_timeline.py 5 2 8 || exit 1
echo done > $out/done
