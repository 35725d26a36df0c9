set -o pipefail
# round 2 (session 3): sustained rate over a long serial run of 5-batch list launches (vring; lean path 13)
out=gpurun_out/s2v
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/sustain_vring.txt python -u tools/sustain.py 400 5 0 || exit 1
tools/gpu_step.sh 200 $out/sustain_lean.txt python -u tools/sustain.py 400 5 13 || exit 1
rocm-smi --showpower --showclocks --showtemp > $out/smi.txt 2>&1 || true
