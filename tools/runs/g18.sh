set -o pipefail
mkdir -p gpurun_out/g18
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 gpurun_out/g18/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/g18/pytest.log || exit 1
for p in 0 2 14; do
    tools/gpu_step.sh 120 gpurun_out/g18/p${p}.log rocprofv3 --kernel-trace --stats -d gpurun_out/g18/p${p} -o run --output-format csv -- python3 tools/profile_one.py --path $p --lanes 8 --reps 30 || exit 1
done
tools/gpu_step.sh 120 gpurun_out/g18/tl.log python -u tools/timeline.py --lanes 8 --path 13 || exit 1
tools/gpu_step.sh 120 gpurun_out/g18/pipe.log python -u tools/pipeline.py --path 0 --lanes 8 --depths 1,2,3,4 || exit 1
