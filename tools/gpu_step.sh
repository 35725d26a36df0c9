#!/bin/bash
# Run one GPU step under its own time limit.
#   tools/gpu_step.sh SECONDS LOGFILE cmd args...
# Any non-zero exit stops the caller's script: a fault, abort, segfault or timeout
# (124/134/137/139, >128) exits 99, and an ordinary failure (a pytest assertion, a
# Python traceback in a measurement leg: rc 1) exits 98.  Every run script chains its
# steps with `|| exit 1`, so an A/B matrix whose first leg fails stops at that leg
# instead of running every later one into the same error (round 5's r5h: 24 legs
# failed silently on a loader error).  GPU_STEP_ALLOW_FAIL=1 lets an ordinary failure
# continue, for a leg whose failure is itself the measurement.
limit=$1; log=$2; shift 2
timeout -k 10 "$limit" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc cmd=$*" >> "$log"
if [ $rc -ge 124 ]; then
  echo "[gpu_step] FATAL rc=$rc for: $* -- stopping" >&2
  exit 99
fi
if [ $rc -ne 0 ] && [ "${GPU_STEP_ALLOW_FAIL:-0}" != "1" ]; then
  echo "[gpu_step] FAILED rc=$rc for: $* -- stopping (log: $log)" >&2
  tail -5 "$log" >&2
  exit 98
fi
exit 0
