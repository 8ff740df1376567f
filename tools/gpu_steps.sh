#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first
# step that crashes, aborts or times out (exit >= 124 or a signal), so nothing
# more touches the GPU after a fault.  A plain test failure (exit 1) does not
# stop later steps.  Usage: tools/gpu_steps.sh "secs|name|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "=== stopping after [$name] (rc=$rc)" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
