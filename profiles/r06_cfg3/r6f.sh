set -o pipefail
# round 6 (f): the records instance's boustrophedon deal (odd rounds in reverse workgroup
# order): GPU suite, cfg3 binned and cfg5 gather A/B against the same
# sources without it (build_ab/libenethip_r6nosnake.so) interleaved x3, the cold records
# timeline after it; the PCIe probe (why the small receive kernel is no faster)
out=gpurun_out/r6f
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NEW=$PWD/enet-csharp_amd/libenethip.so
BASE=$PWD/build_ab/libenethip_r6nosnake.so
tools/gpu_step.sh 900 $out/pytest.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0"
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then L=$BASE; else L=$NEW; fi
    ENET_HIP_LIBRARY=$L tools/gpu_step.sh 300 $out/cfg3b_${v}_$rep.json $B --config cfg3 --binned --streams 1 || exit 1
    ENET_HIP_LIBRARY=$L tools/gpu_step.sh 300 $out/cfg3b6_${v}_$rep.json $B --config cfg3 --binned || exit 1
    ENET_HIP_LIBRARY=$L tools/gpu_step.sh 300 $out/gather_${v}_$rep.log python -u tools/gather_bench.py --only gather_binned || exit 1
  done
done
tools/gpu_step.sh 300 $out/bin_timeline_cold.log python -u tools/bin_timeline.py 3 || exit 1
tools/gpu_step.sh 120 $out/pcieprobe.log tools/pcieprobe || exit 1
echo done > $out/done
