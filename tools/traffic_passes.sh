#!/bin/bash
# The three FETCH_SIZE passes whose records bench.py reads (profiles/traffic_*.json), each in
# its own rocprofv3 run, written to OUTDIR with the sha256 of the product library they ran
# (tools/traffic.py, tools/traffic_sum.py).  Copy them to profiles/ only from a run of the
# library that is committed: bench.py ignores a record of any other build.
#   tools/traffic_passes.sh OUTDIR
out=$1
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/cfg2_fetch -o run --output-format csv \
  -- python3 tools/profile_one.py --reps 20 --probe --list 5 --wgs 2 > $out/cfg2_fetch.log 2>&1
python3 tools/traffic.py $out/cfg2_fetch 78643200 5 $out/traffic_cfg2.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/cfg3b_fetch -o run --output-format csv \
  -- python3 tools/profile_one.py --config cfg3 --binned --reps 8 --probe > $out/cfg3b_fetch.log 2>&1
python3 tools/traffic_sum.py $out/cfg3b_fetch --bytes 192275835 --calls 8 --probe-bytes 192275824 \
  --what "cfg3 binned (enet_hip_crc32_batch_device_binned, default: one launch, the local-tile records instance, 4 lanes)" --binned \
  --out $out/traffic_cfg3_binned.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/cfg5_fetch -o run --output-format csv \
  -- python3 tools/gather_bench.py --only gather_binned --reps 8 --probe 4 > $out/cfg5_fetch.log 2>&1
python3 tools/traffic_sum.py $out/cfg5_fetch --bytes 274857984 --calls 12 --probe-bytes 274857984 \
  --what "cfg5 binned gather (enet_hip_crc32_gather_binned_device, default: local-tile segment pass, one-pass join)" --binned \
  --out $out/traffic_cfg5_binned.json
