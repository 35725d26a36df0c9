set -o pipefail
# round 2 (session 3): the default bench (200 steps) against stream count; the driver form beside it
out=gpurun_out/s2u
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for s in 6 4 2 3; do
  tools/gpu_step.sh 200 $out/steps200_s$s.json python bench.py --no-cpu-baseline --streams $s || exit 1
done
tools/gpu_step.sh 200 $out/steps200_s4_wgs1.json python bench.py --no-cpu-baseline --streams 4 --wgs 1 || exit 1
tools/gpu_step.sh 200 $out/steps20_s6.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh 200 $out/steps20_s4_wgs1.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --streams 4 --wgs 1 || exit 1
tools/gpu_step.sh 200 $out/steps60_s6.json python bench.py --steps 60 --warmup 5 --no-cpu-baseline || exit 1
