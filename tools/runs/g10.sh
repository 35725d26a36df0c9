set -o pipefail
mkdir -p gpurun_out/g10
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 0 2 14; do
  for l in 4 8; do
    tools/gpu_step.sh 120 gpurun_out/g10/p${p}_l${l}.log rocprofv3 --kernel-trace --stats -d gpurun_out/g10/p${p}_l${l} -o run --output-format csv -- python3 tools/profile_one.py --path $p --lanes $l --reps 30 || exit 1
  done
done
