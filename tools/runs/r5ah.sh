set -o pipefail
# round 5 (ah): the per-call stamp + send bench with its stamps checked against the oracle
out=gpurun_out/r5ah
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
UDP_BENCH_SEND_CALLS=1 tools/gpu_step.sh 300 $out/send_calls.log python -u tools/udp_bench.py || exit 1
echo done > $out/done
