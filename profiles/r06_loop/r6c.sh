set -o pipefail
# round 6 (c): the vring ring loop with one exit (the 8 v_readfirstlane latch
# copies gone): GPU suite on the new build, then A/B against the same sources with the old
# two-exit loop (build_ab/libenethip_r6base.so), interleaved x3 on one box; SQ counters of the
# new build; the receive call's cost against the CPU callback at 8-256 DGRAMs per call
#  and a runtime trace of it
out=gpurun_out/r6c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NEW=$PWD/enet-csharp_amd/libenethip.so
BASE=$PWD/build_ab/libenethip_r6base.so
tools/gpu_step.sh 900 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then L=$BASE; else L=$NEW; fi
    ENET_HIP_LIBRARY=$L tools/gpu_step.sh 300 $out/drv_${v}_$rep.json $B || exit 1
    ENET_HIP_LIBRARY=$L tools/gpu_step.sh 300 $out/ser_${v}_$rep.json $B --streams 1 --sustain-ms 0 || exit 1
    ENET_HIP_LIBRARY=$L tools/gpu_step.sh 300 $out/one_${v}_$rep.json $B --list 0 --streams 1 --sustain-ms 0 || exit 1
    ENET_HIP_LIBRARY=$L tools/gpu_step.sh 300 $out/ver_${v}_$rep.log python -u tools/verify_bench.py --list 20 || exit 1
  done
done
for v in base new; do
  if [ $v = base ]; then L=$BASE; else L=$NEW; fi
  ENET_HIP_LIBRARY=$L tools/gpu_step.sh 300 $out/def_${v}.json python bench.py --no-cpu-baseline || exit 1
done
bash tools/pmc_mix.sh $out/pmc_new --list 5 --reps 20 > $out/pmc_new.log 2>&1 || exit 1
python3 tools/pmc_summary.py $out/pmc_new vring > $out/pmc_new_summary.txt || exit 1
UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,32,64,128,256 UDP_BENCH_CALL_MODES=gpu,callback,recv \
  tools/gpu_step.sh 300 $out/rx_calls.log python -u tools/udp_bench.py || exit 1
UDP_BENCH_CALLS=1 UDP_BENCH_KS=8,256 UDP_BENCH_CALL_MODES=gpu timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats \
  -d $out/rx_trace -o run --output-format csv -- python3 tools/udp_bench.py > $out/rx_trace.log 2>&1 || exit 1
echo done > $out/done
