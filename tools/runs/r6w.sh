set -o pipefail
# round 6 (w): the plain gather entry (one lane per DGRAM) against the binned gather on cfg5
out=gpurun_out/r6w
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/gather_both.log python -u tools/gather_bench.py || exit 1
touch $out/done
