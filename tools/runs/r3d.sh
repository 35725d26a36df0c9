set -o pipefail
# round 3 (d): catch the intermittent unset groups at 2 workgroups per CU with the trace instance
out=gpurun_out/r3d
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/trace_dbg_l8.log python -u tools/dbg/trace_dbg.py 8 0 80 || exit 1
tools/gpu_step.sh 300 $out/trace_dbg_l4_p21.log python -u tools/dbg/trace_dbg.py 4 21 80 || exit 1
