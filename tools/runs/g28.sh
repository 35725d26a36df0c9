set -o pipefail
out=gpurun_out/g28
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in 0 64 0 64; do
    tools/gpu_step.sh 120 $out/a${a}.log rocprofv3 --kernel-trace --stats -d $out/a${a}_$RANDOM -o run --output-format csv -- python3 tools/profile_one.py --path 13 --lanes 8 --ablate $a --reps 30 || exit 1
done
tools/gpu_step.sh 200 $out/pipe0.log python -u tools/pipeline.py --path 13 --lanes 8 --depths 1,6 || exit 1
tools/gpu_step.sh 200 $out/pipe64.log python -u tools/pipeline.py --path 13 --lanes 8 --ablate 64 --depths 1,6 || exit 1
