set -o pipefail
# round 2: stream-kernel zero-stage fix + batch-list vring -- parity, then benches
out=gpurun_out/r2r
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/listprobe.log python -u tools/listprobe.py || exit 1
grep -q "^done" $out/listprobe.log || exit 1
tools/gpu_step.sh 300 $out/pytest_new.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "empty or vring or batch_list" || exit 1
grep -q " passed" $out/pytest_new.log || exit 1
grep -q "failed\|Timeout" $out/pytest_new.log && exit 1
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
tools/gpu_step.sh 300 $out/bench_list5.json python bench.py --list 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/bench_list5_s1.json python bench.py --list 5 --streams 1 --no-cpu-baseline || exit 1
