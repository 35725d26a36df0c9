set -o pipefail
mkdir -p gpurun_out/g12
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in 0 1 2 3; do
    tools/gpu_step.sh 120 gpurun_out/g12/a${a}.log rocprofv3 --kernel-trace --stats -d gpurun_out/g12/a${a} -o run --output-format csv -- python3 tools/profile_one.py --path 13 --lanes 8 --ablate $a --reps 30 || exit 1
done
