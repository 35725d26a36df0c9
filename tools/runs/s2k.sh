set -o pipefail
# round 2: probe kernels with a CRC-like fold (32 LDS lookups per 32 B), depth 1 vs prefetch
out=gpurun_out/s2k
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SP_CFGS=9,18,21,26,27,28,29,30,31,32,33 tools/gpu_step.sh 300 $out/probe.txt python -u tools/streamprobe.py probe || exit 1
