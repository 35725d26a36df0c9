set -o pipefail
out=gpurun_out/g32
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest_binned.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k binned --timeout 120 --timeout-method thread || exit 1
grep -q " passed" $out/pytest_binned.log || exit 1
grep -q "failed" $out/pytest_binned.log && exit 1
tools/gpu_step.sh 400 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for l in 4 8; do
  tools/gpu_step.sh 200 $out/cfg3_l$l.json python bench.py --config cfg3 --lanes $l --no-cpu-baseline --steps 100 || exit 1
  tools/gpu_step.sh 200 $out/cfg3_binned_l$l.json python bench.py --config cfg3 --lanes $l --binned --no-cpu-baseline --steps 100 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/cfg3_binned_trace -o run --output-format csv -- python3 bench.py --config cfg3 --lanes 8 --binned --streams 1 --steps 100 --no-cpu-baseline > $out/cfg3_binned_rocprof.json 2> $out/cfg3_binned_rocprof.err || exit 1
