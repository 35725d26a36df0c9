set -o pipefail
out=gpurun_out/g22
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 200 $out/pipe.log python -u tools/pipeline.py --path 0 --lanes 8 --depths 1,4,6,8 || exit 1
tools/gpu_step.sh 200 $out/pipe_prio.log python -u tools/pipeline.py --path 0 --lanes 8 --ablate 8 --depths 1,4,8 || exit 1
for a in 0 8; do
    tools/gpu_step.sh 120 $out/a${a}.log rocprofv3 --kernel-trace --stats -d $out/a${a} -o run --output-format csv -- python3 tools/profile_one.py --path 13 --lanes 8 --ablate $a --reps 30 || exit 1
done
