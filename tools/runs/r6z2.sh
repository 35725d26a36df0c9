set -o pipefail
# round 6: final validation of the committed tree -- the whole GPU suite (C host included),
# smoke, the driver's bench command, and the driver's 2-rank launcher form on this one GPU
# (two ranks sharing the device: checks the distributed path, not a scaling number)
out=gpurun_out/r6z2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
sha256sum enet-csharp_amd/libenethip.so > $out/lib_sha.txt
tools/gpu_step.sh 900 $out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit 1
tools/gpu_step.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 $out/bench_ranks2.json python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
touch $out/done
