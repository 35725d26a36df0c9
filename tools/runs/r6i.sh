set -o pipefail
# round 6 (i): the deal probe -- cfg3's binned order read under the global rank-interleaved
# deal against per-workgroup local tiles (tools/dealprobe.hip)
out=gpurun_out/r6i
mkdir -p $out
tools/gpu_step.sh 120 $out/dealprobe.txt ./tools/dealprobe 262144
