set -o pipefail
mkdir -p gpurun_out/g4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 gpurun_out/g4/dma.log python -u tools/dmabench.py || exit 1
tools/gpu_step.sh 200 gpurun_out/g4/prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/g4/prof -o run --output-format csv -- python3 tools/dmabench.py || exit 1
