set -o pipefail
mkdir -p gpurun_out/g19
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 gpurun_out/g19/pytest.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lean or cfg2 or cfg3 or verify or golden" || exit 1
grep -q " passed" gpurun_out/g19/pytest.log || exit 1
for a in 0 1 5; do
    tools/gpu_step.sh 120 gpurun_out/g19/a${a}.log rocprofv3 --kernel-trace --stats -d gpurun_out/g19/a${a} -o run --output-format csv -- python3 tools/profile_one.py --path 13 --lanes 8 --ablate $a --reps 30 || exit 1
done
tools/gpu_step.sh 120 gpurun_out/g19/tl.log python -u tools/timeline.py --lanes 8 --path 13 || exit 1
