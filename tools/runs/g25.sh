set -o pipefail
out=gpurun_out/g25
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for s in 4 6 3 8 4 6; do
  tools/gpu_step.sh 200 $out/b_s$s.json python bench.py --no-cpu-baseline --streams $s || exit 1
  grep metric $out/b_s$s.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('streams', $s, d['value'], d['ms_per_step'])" >> $out/summary.txt
done
for s in 4 6; do
  tools/gpu_step.sh 200 $out/b_r6_s$s.json python bench.py --no-cpu-baseline --streams $s --rotate 6 || exit 1
  grep metric $out/b_r6_s$s.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('rot6 streams', $s, d['value'], d['ms_per_step'])" >> $out/summary.txt
done
