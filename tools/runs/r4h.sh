set -o pipefail
# round 3 (4h): stress of the round-3 kernel paths (records instance, binned gather, verify), 25 repeats each
out=gpurun_out/r4h
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/stress_r3.log python -u tools/dbg/stress_r3.py 25 || exit 1
