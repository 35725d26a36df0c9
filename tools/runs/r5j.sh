set -o pipefail
# round 5 (j): the split gather join (pre-join beside the binning tiles, post-join per
# segment) on the GPU -- parity, A/B against the VALU-cut library without it and against
# the one-pass join in the same diagnostics build; VERDICT r4 #6 one cfg4 shard per N
# with its kernel trace; VERDICT r4 #3 VALU per byte and the sustained rate; the cfg3
# lanes x workgroups sweep; ADVICE r4 tiny fragment batches against a large claim space
out=gpurun_out/r5j
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_step.sh 600 $out/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread -k "gather or harness or fragments or dynamic_rounds" tests/test_gpu_parity.py tests/test_gpu_harness.py tests/test_gpu_fragments.py || exit 1
grep -q " passed" $out/pytest.log || exit 1
grep -q "FAILED" $out/pytest.log && exit 1
for rep in 1 2 3; do
  for v in r5b r5c; do
    ENET_HIP_LIBRARY=$PWD/build_ab/libenethip_$v.so tools/gpu_step.sh 300 $out/gather_${v}_$rep.log python tools/gather_bench.py --only gather_binned --reps 50 || exit 1
  done
  tools/gpu_step.sh 300 $out/onepass_$rep.log python tools/gather_bench.py --only gather_binned --reps 50 --ablate 4194304 || exit 1
done
tools/gpu_step.sh 300 $out/rocprof_gather.log rocprofv3 --kernel-trace --stats -d $out/prof_gather -o run --output-format csv -- python tools/gather_bench.py --only gather_binned --reps 24 || exit 1
for N in 1 2 4 8; do
  tools/gpu_step.sh 300 $out/shard_0of$N.json python bench.py --config cfg4 --shard 0/$N --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 300 $out/shard_0of${N}_rocprof.log rocprofv3 --kernel-trace --stats -d $out/prof_shard$N -o run --output-format csv -- python bench.py --config cfg4 --shard 0/$N --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
bash tools/pmc_mix.sh $out/pmc_cfg2 --list 5 --reps 20 > $out/pmc_cfg2.log 2>&1 || exit 1
tools/gpu_step.sh 300 $out/sustain_vring.log python tools/sustain.py --kernel vring --launches 3000 || exit 1
for l in 4 8; do for w in 1 2; do
  tools/gpu_step.sh 300 $out/cfg3b_l${l}_w$w.json python bench.py --config cfg3 --binned --lanes $l --wgs $w --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done; done
for m in 1024 1025; do
  tools/gpu_step.sh 300 $out/frag_tiny_$m.log python tools/frag_bench.py --messages $m --words 2 --first 1 --reps 50 || exit 1
done
for m in 1032 1033; do
  tools/gpu_step.sh 300 $out/frag_small_$m.log python tools/frag_bench.py --messages $m --words 2 --first 64 --reps 50 || exit 1
done
echo done > $out/done
