set -o pipefail
# round 2: DMA pattern a64 + lean geometry sweep (W x NB)
out=gpurun_out/r2b
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/dma.log python -u tools/dmabench.py || exit 1
for p in 13 14 15 16; do
  tools/gpu_step.sh 200 $out/pipe_p$p.log python -u tools/pipeline.py --path $p --lanes 8 --depths 1,6 || exit 1
done
