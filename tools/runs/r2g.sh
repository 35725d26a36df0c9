set -o pipefail
# round 2: vring with explicit counted waits -- parity, then timing
out=gpurun_out/r2g
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for l in 8 4; do
  tools/gpu_step.sh 200 $out/pipe_l${l}.log python -u tools/pipeline.py --path 0 --lanes $l --depths 1,2,6 || exit 1
  tools/gpu_step.sh 200 $out/pipe_l${l}_2wg.log python -u tools/pipeline.py --path 0 --lanes $l --ablate 512 --depths 1,2,6 || exit 1
done
