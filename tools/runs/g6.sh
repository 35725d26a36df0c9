set -o pipefail
mkdir -p gpurun_out/g6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 120 gpurun_out/g6/tl8.log python -u tools/timeline.py --lanes 8 || exit 1
tools/gpu_step.sh 120 gpurun_out/g6/tl4.log python -u tools/timeline.py --lanes 4 || exit 1
tools/gpu_step.sh 300 gpurun_out/g6/mix.log bash tools/pmc_mix.sh gpurun_out/g6/pmc --path 13 --lanes 8 --reps 5 || exit 1
python3 tools/pmc_summary.py gpurun_out/g6/pmc crc32 > gpurun_out/g6/pmc_summary.txt
