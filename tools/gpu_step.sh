#!/bin/bash
# Run one GPU step under its own time limit; stop the whole GPU call on a fault,
# abort, segfault or timeout (exit 124/134/137/139 or >128), continue on ordinary
# failures (e.g. a pytest assertion, exit 1).
#   tools/gpu_step.sh SECONDS LOGFILE cmd args...
limit=$1; log=$2; shift 2
timeout -k 10 "$limit" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc cmd=$*" >> "$log"
if [ $rc -ge 124 ]; then
  echo "[gpu_step] FATAL rc=$rc for: $* -- stopping" >&2
  exit 99
fi
exit 0
