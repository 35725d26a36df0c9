set -o pipefail
# round 3 (4g): rocprof kernel trace of the cfg3 binned entry (bin kernel vs records kernel)
out=gpurun_out/r4g
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/cfg3b_trace -o run --output-format csv \
  -- python3 tools/profile_one.py --config cfg3 --binned --reps 20 > $out/cfg3b_trace.log 2>&1 || exit 1
