set -o pipefail
# round 2 (session 4): vring with workgroup walks (paths 19/20) -- parity, then bench vs path 0
out=gpurun_out/s3b
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "many_groups or batch_list" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
for p in 0 19 20; do
  tools/gpu_step.sh 200 $out/p${p}_driver.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --path $p || exit 1
  tools/gpu_step.sh 200 $out/p${p}_l20.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --path $p --list 20 --rotate 20 --streams 1 || exit 1
done
