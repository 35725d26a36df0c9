set -o pipefail
# round 4 (ap): range coder model layout (lane-major vs symbol-major) at 16 and 8 lanes per wave
out=gpurun_out/r4ap
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/rc_layout.log python3 -u tools/rc_bench.py --sweep 16:16:0,16:16:1,8:32:0,8:32:1,64:4:1,16:16:0,16:16:1 || exit 1
echo done > $out/done
