set -o pipefail
# round 2: DMA access-pattern ceilings (dmabench lean-like patterns, nt policy)
# and the lean kernel with nt data loads vs default
out=gpurun_out/r2a
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh 200 $out/dma.log python -u tools/dmabench.py || exit 1
for a in 0 256 0 256; do
  tools/gpu_step.sh 200 $out/pipe_a$a.log python -u tools/pipeline.py --path 13 --lanes 8 --ablate $a --depths 1,6 || exit 1
done
