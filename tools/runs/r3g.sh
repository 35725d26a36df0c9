set -o pipefail
# round 3 (g): blocking context stream (the stress "unwritten" race) + vring receive verify:
# stress (all variants), GPU suite, verify bench, tail-first A/B benches, per-kernel rocprof + FETCH
out=gpurun_out/r3g
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/stress.log python -u tools/dbg/stress.py 25 || exit 1
tools/gpu_step.sh 1000 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" $out/pytest.log || exit 1
tools/gpu_step.sh 300 $out/verify_bench.log python -u tools/verify_bench.py || exit 1
tools/gpu_step.sh 300 $out/verify_bench_list20.log python -u tools/verify_bench.py --list 20 || exit 1
tools/gpu_step.sh 300 $out/verify_bench_lean.log python -u tools/verify_bench.py --path 13 || exit 1
OUT=$out bash tools/runs/r3f.sh || exit 1