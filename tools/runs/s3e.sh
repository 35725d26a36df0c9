set -o pipefail
# round 2 (session 4): receive-verify batch lists (lean MODE 1 list instance) -- parity, then throughput
out=gpurun_out/s3e
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pytest.log python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "verify" || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "failed\|Timeout" $out/pytest.log && exit 1
for l in 0 4 8; do
  tools/gpu_step.sh 200 $out/verify_l$l.json python -u tools/verify_bench.py --lanes $l --list 5 || exit 1
done
tools/gpu_step.sh 200 $out/verify_l4_list20.json python -u tools/verify_bench.py --lanes 4 --list 20 --rotate 20 || exit 1
