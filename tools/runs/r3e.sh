set -o pipefail
# round 3 (e): the intermittent unset groups at 2 workgroups per CU -- stress with a
# never-written sentinel (asm slot-counter atomic), then end-record instrumentation (TR 2)
out=gpurun_out/r3e
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/stress.log python -u tools/dbg/stress.py 25 || exit 1
tools/gpu_step.sh 300 $out/tr2_l8.log python -u tools/dbg/tr2_dbg.py 8 100 || exit 1
tools/gpu_step.sh 300 $out/tr2_l4.log python -u tools/dbg/tr2_dbg.py 4 100 || exit 1
