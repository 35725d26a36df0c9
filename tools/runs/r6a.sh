set -o pipefail
# round 6 (a): the shared-boundary-line probe.  cfg2 5-batch lists, serial
# (--streams 1), window order (path 0) against tail-first (path 21: the boundary line is read by
# both neighbours in adjacent steps), with and without the fold's lookups (--ablate 4096), at one
# and two workgroups per CU; each leg timed by the bench's HIP-event region and its FETCH_SIZE
# from its own rocprofv3 pass.  Any failing leg stops the script (tools/gpu_step.sh).
out=gpurun_out/r6a
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --gpus 1 --steps 20 --warmup 5 --streams 1 --no-cpu-baseline --sustain-ms 0"
for rep in 1 2; do
  for w in 1 2; do
    for pa in "0 0" "0 4096" "0 38912" "21 0" "21 4096"; do
      set -- $pa
      tools/gpu_step.sh 300 $out/b_p$1_a$2_w${w}_$rep.json $B --wgs $w --path $1 --ablate $2 || exit 1
    done
  done
done
for w in 1 2; do
  for pa in "0 0" "0 4096" "0 38912" "21 0" "21 4096"; do
    set -- $pa
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/f_p$1_a$2_w$w -o run --output-format csv \
      -- python3 tools/profile_one.py --reps 20 --probe --list 5 --wgs $w --path $1 --ablate $2 > $out/f_p$1_a$2_w$w.log 2>&1 || exit 1
    python3 tools/traffic.py $out/f_p$1_a$2_w$w 78643200 5 $out/t_p$1_a$2_w$w.json || exit 1
  done
done
echo done > $out/done
