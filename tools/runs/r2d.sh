set -o pipefail
# round 2: vring kernel -- GPU parity suite, then serial/overlapped timing vs the lean kernel
out=gpurun_out/r2d
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
tools/gpu_step.sh 200 $out/pipe_p0.log python -u tools/pipeline.py --path 0 --lanes 8 --depths 1,6 || exit 1
tools/gpu_step.sh 200 $out/pipe_p13.log python -u tools/pipeline.py --path 13 --lanes 8 --depths 1,6 || exit 1
tools/gpu_step.sh 200 $out/pipe_p0b.log python -u tools/pipeline.py --path 0 --lanes 4 --depths 1,6 || exit 1
