set -o pipefail
# round 5 (a): the loader-wave ring probe beside the product bench on one box
out=gpurun_out/r5a
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 300 $out/ringprobe.log tools/ringprobe || exit 1
tools/gpu_step.sh 300 $out/bench_driver.json python bench.py --steps 20 --warmup 5 || exit 1
echo done > $out/done
