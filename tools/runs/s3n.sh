set -o pipefail
# round 2 (session 4): length-binned records on the lean (path 0) vs vring (17) kernel, 4 and 8 lanes: cfg3 and cfg5 gather
out=gpurun_out/s3n
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 0 17; do for l in 4 8; do
  tools/gpu_step.sh 200 $out/cfg3_p${p}_l${l}.json python bench.py --config cfg3 --binned --lanes $l --path $p --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/gather_p${p}_l${l}.json python -u tools/gather_bench.py --lanes $l --path $p || exit 1
done; done
