#!/bin/bash
# Run GPU steps in order, each under its own time limit. Test failures (exit 1) continue to the
# next step; any crash / abort / timeout (exit >= 2: 124, 134, 137, 139, ...) ends the session.
# usage: tools/gpu_session.sh "<name>|<seconds>|<command>" ...
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then
    echo "=== stopping session after [$name] (rc=$rc)"
    exit $rc
  fi
done
exit 0
