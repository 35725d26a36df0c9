set -o pipefail
# round 2 (session 3): burst probes (D stages per packet per burst, W waves per CU), with and without a fold;
# config 1 on the box host
out=gpurun_out/s2p
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SP_CFGS=9,11,42,43,44,45,46,47,48,49,50,51,52,53 tools/gpu_step.sh 300 $out/probe.txt python -u tools/streamprobe.py probe || exit 1
gcc -O2 -o $out/cfg1_loop tools/cfg1_loop.c -ldl && ($out/cfg1_loop enet-csharp_amd/libenethip.so oracle/lib/liboracle.so 1024 256 3.0 > $out/cfg1.json 2>&1; lscpu > $out/lscpu.txt) || exit 1
