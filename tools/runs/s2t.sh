set -o pipefail
# round 2 (session 3): driver-form bench (--steps 20): lean vs vring lists, list length x streams
out=gpurun_out/s2t
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 0 17; do
  tools/gpu_step.sh 200 $out/p${p}_l5.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --path $p || exit 1
  tools/gpu_step.sh 200 $out/p${p}_l10s2.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --path $p --list 10 --rotate 10 --streams 2 || exit 1
  tools/gpu_step.sh 200 $out/p${p}_l20.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --path $p --list 20 --rotate 20 --streams 1 || exit 1
  tools/gpu_step.sh 200 $out/p${p}_l4s5.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --path $p --list 4 --streams 5 || exit 1
  tools/gpu_step.sh 200 $out/p${p}_l5b.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --path $p || exit 1
done
