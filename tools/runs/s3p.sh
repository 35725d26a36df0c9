set -o pipefail
# round 2 (session 4): partial lgkmcnt(4) waits in the vring fold -- parity on the variant, A/B on one box
out=gpurun_out/s3p
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  tools/gpu_step.sh 200 $out/base_$r.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $out/lgkm4_$r.json python tools/ablib.py tools/libenethip_lgkm4.so bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
tools/gpu_step.sh 200 $out/base_l20.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --list 20 --rotate 20 --streams 1 || exit 1
tools/gpu_step.sh 200 $out/lgkm4_l20.json python tools/ablib.py tools/libenethip_lgkm4.so bench.py --steps 20 --warmup 5 --no-cpu-baseline --list 20 --rotate 20 --streams 1 || exit 1
