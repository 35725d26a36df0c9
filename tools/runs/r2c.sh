set -o pipefail
# round 2: pipebench -- lean memory pipeline variants (ring depth, table layout, alignment)
out=gpurun_out/r2c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/pb.log python -u tools/pipebench.py ${PB_CFGS:-} || exit 1
