set -o pipefail
# round 4 (x): single-batch checksum and verify -- kernel durations (rocprof) beside the
# per-call serial times, and the list forms
out=gpurun_out/r4x
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/verify_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_verify -o run -- python3 -u tools/verify_bench.py --reps 50 --list 20 || exit 1
tools/gpu_step.sh 300 $out/bench_l0_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_l0 -o run -- python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --sustain-ms 0 --list 0 --streams 1 || exit 1
echo done > $out/done
