set -o pipefail
# round 2 (session 4): SQ instruction-mix / stall / LDS counters of the final vring (8 lanes, 5-batch lists, 2 wg/CU)
out=gpurun_out/s3s
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_mix.sh $out --reps 20 --list 5 --wgs 2 > $out/pmc.log 2>&1 || exit 1
