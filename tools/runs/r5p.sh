set -o pipefail
# round 5 (p): single-batch launches on the cheaper fold -- lanes x workgroups per CU for
# the checksum (bench --list 0) and the verify (verify_bench), interleaved 2x
out=gpurun_out/r5p
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for l in 8 4; do for w in 1 2; do
    tools/gpu_step.sh 300 $out/single_l${l}_w${w}_$rep.json python bench.py --list 0 --lanes $l --wgs $w --steps 20 --warmup 5 --no-cpu-baseline --sustain-ms 0 || exit 1
    tools/gpu_step.sh 300 $out/verify_l${l}_w${w}_$rep.log python -u tools/verify_bench.py --lanes $l --wgs $w --list 20 || exit 1
  done; done
done
echo done > $out/done
