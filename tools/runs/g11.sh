set -o pipefail
mkdir -p gpurun_out/g11
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 gpurun_out/g11/pytest.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread || exit 1
for p in 13 14; do
  for l in 4 8; do
    tools/gpu_step.sh 120 gpurun_out/g11/p${p}_l${l}.log rocprofv3 --kernel-trace --stats -d gpurun_out/g11/p${p}_l${l} -o run --output-format csv -- python3 tools/profile_one.py --path $p --lanes $l --reps 30 || exit 1
  done
done
tools/gpu_step.sh 120 gpurun_out/g11/tl8.log python -u tools/timeline.py --lanes 8 || exit 1
