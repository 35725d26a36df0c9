set -o pipefail
# round 6 (u): closing evidence of the final build (after the fragment clash kernel), part 1:
# -m gpu, smoke, the three FETCH_SIZE passes of this build, bench lines (driver form x2, default)
out=gpurun_out/r6u
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
sha256sum enet-csharp_amd/libenethip.so > $out/lib_sha.txt
tools/gpu_step.sh 900 $out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
tools/gpu_step.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
grep -q "smoke ok" $out/smoke.log || exit 1
bash tools/traffic_passes.sh $out || exit 1
tools/gpu_step.sh 300 $out/bench_driver_1.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_driver_2.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_default.json python bench.py || exit 1
echo done > $out/done
