set -o pipefail
# round 4 (ba): cfg1 loopback echo on the GPU box's host CPU with the carry-less-multiply
# callback (tools/cfg1_loop.c; no GPU use)
out=gpurun_out/r4ba
mkdir -p $out
for rep in 1 2 3; do
  timeout -k 10 120 ./tools/cfg1_loop_bin enet-csharp_amd/libenethip.so oracle/lib/liboracle.so 1024 256 2.0 > $out/cfg1_$rep.json || exit 1
done
grep -o "pclmulqdq" /proc/cpuinfo | head -1 > $out/cpu_has_pclmul.txt || true
echo done > $out/done
