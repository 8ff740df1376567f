#!/bin/bash
# Run GPU steps one after another on the gpurun box, each under its own time
# limit, logging to gpurun_out/<name>.log.  Stops at the first failing step
# (fault, abort, timeout) so nothing more touches the GPU after trouble.
#
#   bash tools/gpu_steps.sh "SECONDS|name|command" ["SECONDS|name|command" ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"
  name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s) $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start )) s"
  tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    echo "=== stopping after failed step $name"
    exit $rc
  fi
done
echo "=== all steps ok"
