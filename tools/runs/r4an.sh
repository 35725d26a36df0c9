set -o pipefail
# round 4 (an): range coder lanes per wave x waves per CU (diagnostics sweep), compressed
# bytes checked against the first configuration, round trip checked each time
out=gpurun_out/r4an
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 400 $out/rc_sweep.log python3 -u tools/rc_bench.py --sweep 64:4,32:8,16:16,8:32,64:8,32:16,16:32,4:32,64:4 || exit 1
echo done > $out/done
