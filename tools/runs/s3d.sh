set -o pipefail
# round 2 (session 4): receive-verify throughput (lean MODE 1) vs checksum on cfg2-shaped DGRAMs
out=gpurun_out/s3d
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for l in 0 4 8; do
  tools/gpu_step.sh 200 $out/verify_l$l.json python -u tools/verify_bench.py --lanes $l || exit 1
done
