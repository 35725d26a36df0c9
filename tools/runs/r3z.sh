set -o pipefail
# round 3 (z): bench.py's multi-rank path on the real GPU engine, launched as the driver launches
# it (torch.distributed.run, one process per rank, gloo barrier / max-over-ranks): 2 ranks sharing
# the box's one GPU (device = LOCAL_RANK mod device count), weak (cfg2) and strong (cfg4) scaling
out=gpurun_out/r3z
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517"
tools/gpu_step.sh 300 $out/dist2_cfg2.json $R bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh 300 $out/dist2_cfg4.json $R bench.py --gpus 2 --config cfg4 --steps 8 --warmup 2 --no-cpu-baseline --sustain-ms 0 || exit 1
tools/gpu_step.sh 300 $out/dist1_cfg2.json python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
