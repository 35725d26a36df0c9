#!/bin/bash
# Kernel time vs batch size (fixed 1200-B packets): separates per-launch fixed
# cost from the streaming rate.  Usage: tools/size_scan.sh "path:lanes" ...
for n in 16384 32768 65536 131072 262144; do
  for cfg in "$@"; do
    p=${cfg%%:*}; l=${cfg##*:}
    echo "== n=$n path=$p lanes=$l"
    python tools/sweep.py --config fixed:$n --paths $p --lanes $l --wgs 1 --steps 30 --rotate 3 | python3 tools/sweep_table.py
  done
done
