set -o pipefail
# round 2 (session 3): driver-form bench with dynamic slots -- workgroups per CU x list length x streams
out=gpurun_out/s2y
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in 1 2; do
  tools/gpu_step.sh 200 $out/w${w}_l20.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --wgs $w --list 20 --rotate 20 --streams 1 || exit 1
  tools/gpu_step.sh 200 $out/w${w}_l10s2.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --wgs $w --list 10 --rotate 10 --streams 2 || exit 1
  tools/gpu_step.sh 200 $out/w${w}_l4s5.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --wgs $w --list 4 --streams 5 || exit 1
  tools/gpu_step.sh 200 $out/w${w}_l5s6.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --wgs $w || exit 1
  tools/gpu_step.sh 200 $out/w${w}_l5s2.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --wgs $w --streams 2 || exit 1
done
