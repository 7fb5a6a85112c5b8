#!/bin/bash
# Run one GPU step under a time limit; abort the whole call on a fault/timeout.
# usage: tools/gpu_check.sh <seconds> <logfile> <cmd...>
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_check] rc=$rc : $*" >> "$log"
if [ $rc -ge 124 ]; then
  echo "[gpu_check] fatal rc=$rc (timeout/signal) -- stopping" >&2
  exit 100
fi
exit 0
