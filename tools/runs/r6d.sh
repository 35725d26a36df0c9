set -o pipefail
# round 6 (d): after removing the closed linear-stream kernel and adding the records kernel's
# trace instance (diagnostics): GPU suite; the cfg3 binned records timeline;
# the launch-cost probe (the receive call's fixed cost); cfg3 binned serial
# lines; the traffic passes of this build
out=gpurun_out/r6d
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 900 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
tools/gpu_step.sh 300 $out/bin_timeline.log python -u tools/bin_timeline.py 3 || exit 1
tools/gpu_step.sh 120 $out/launchprobe.log tools/launchprobe || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
tools/gpu_step.sh 300 $out/cfg3b_ser_1.json $B --config cfg3 --binned --streams 1 || exit 1
tools/gpu_step.sh 300 $out/cfg3b_ser_2.json $B --config cfg3 --binned --streams 1 || exit 1
tools/gpu_step.sh 120 $out/alignprobe_cfg3_cold.txt ./tools/alignprobe_bin 262144 || exit 1
bash tools/traffic_passes.sh $out || exit 1
sha256sum enet-csharp_amd/libenethip.so > $out/lib_sha.txt
echo done > $out/done
