#!/bin/bash
# Run one gpurun call, retrying ONLY when gpurun reports that nothing ran
# (no free box / transient infrastructure failure); any real result -- pass
# or fail -- ends the loop.  Usage: bash tools/gpu_retry.sh OUT TIMEOUT SCRIPT
out="$1"; lim="$2"; script="$3"
for i in 1 2 3 4 5 6 7 8; do
  timeout $((lim + 900)) /usr/local/graft/bin/gpurun --timeout "$lim" -- bash "$script" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient\|no free box" "$out" && ! grep -q "=== \[" "$out"; then sleep 150; continue; fi
  exit $rc
done
exit $rc
