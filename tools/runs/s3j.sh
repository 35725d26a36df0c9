set -o pipefail
# round 2 (session 4): lanes x workgroups per CU with the hoisted lane constants
out=gpurun_out/s3j
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for l in 4 8; do for w in 1 2; do
  tools/gpu_step.sh 200 $out/l${l}_w${w}_driver.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --lanes $l --wgs $w || exit 1
  tools/gpu_step.sh 200 $out/l${l}_w${w}_l20.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --lanes $l --wgs $w --list 20 --rotate 20 --streams 1 || exit 1
done; done
