set -o pipefail
mkdir -p gpurun_out/g17
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in 0 1 5 16 17 21; do
    tools/gpu_step.sh 120 gpurun_out/g17/a${a}.log rocprofv3 --kernel-trace --stats -d gpurun_out/g17/a${a} -o run --output-format csv -- python3 tools/profile_one.py --path 13 --lanes 8 --ablate $a --reps 30 || exit 1
done
tools/gpu_step.sh 120 gpurun_out/g17/tl_a21.log python -u tools/timeline.py --lanes 8 --path 13 --ablate 21 || exit 1
tools/gpu_step.sh 120 gpurun_out/g17/tl_a16.log python -u tools/timeline.py --lanes 8 --path 13 --ablate 16 || exit 1
