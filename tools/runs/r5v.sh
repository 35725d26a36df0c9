set -o pipefail
# round 5 (v): where a small receive call's time goes -- kernel and HIP API trace of the
# per-call bench (in place form)
out=gpurun_out/r5v
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
UDP_BENCH_CALLS=1 tools/gpu_step.sh 400 $out/prof_calls.log rocprofv3 --kernel-trace --hip-trace --stats -d $out/prof -o run -- python3 -u tools/udp_bench.py || exit 1
echo done > $out/done
