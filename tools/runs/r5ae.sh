set -o pipefail
# round 5 (ae): per-call receive cost with the lean kernel (path 13) verifying the pinned
# arena in place, against the default vring path, and the kernel trace of both
out=gpurun_out/r5ae
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
UDP_BENCH_CALLS=1 tools/gpu_step.sh 300 $out/calls_vring.log python -u tools/udp_bench.py || exit 1
UDP_BENCH_CALLS=1 UDP_BENCH_PATH=13 tools/gpu_step.sh 300 $out/calls_lean.log python -u tools/udp_bench.py || exit 1
UDP_BENCH_CALLS=1 UDP_BENCH_PATH=13 tools/gpu_step.sh 400 $out/prof_lean.log rocprofv3 --kernel-trace --stats -d $out/prof_lean -o run --output-format csv -- python3 -u tools/udp_bench.py || exit 1
echo done > $out/done
