#!/bin/bash
# gpurun with retries on infrastructure-side transients (no box, box lost while
# being prepared, back-off); a run that reached the box is never repeated.
# usage: tools/gpr.sh <timeout> <log> '<command>'
t=$1; log=$2; cmd=$3
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  if grep -q "status=transient\|no free box\|backing off\|retry in" "$log" && ! grep -q "status=ok\|status=fail" "$log"; then
    sleep 75
    continue
  fi
  break
done
grep -v "every call" "$log" | tail -3
