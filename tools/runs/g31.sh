set -o pipefail
out=gpurun_out/g31
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# host toolchain probe for the C# baseline and the host CPU model
{ for t in dotnet mono csc mcs; do printf '%s: ' $t; command -v $t || echo absent; done
  lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket"; } > $out/host_probe.txt 2>&1
tools/gpu_step.sh 300 $out/bench.json python bench.py || exit 1
tools/gpu_step.sh 300 $out/bench_streams1.json python bench.py --streams 1 --no-cpu-baseline || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/serial_trace -o run --output-format csv -- python3 bench.py --streams 1 --steps 200 --warmup 20 --no-cpu-baseline > $out/serial_under_rocprof.json 2> $out/serial_under_rocprof.err || exit 1
