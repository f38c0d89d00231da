#!/bin/bash
# Same-box A/B/C... over environment settings, interleaved so drift cancels.
# usage: tools/env_ab.sh ROUNDS "NAME1|ENV1" "NAME2|ENV2" ... -- [bench args]
mkdir -p gpurun_out
n=$1; shift
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" = "--" ] && shift
for i in $(seq "$n"); do
  for spec in "${specs[@]}"; do
    name="${spec%%|*}"; envs="${spec#*|}"
    env $envs timeout -k 10 150 python bench.py --fit-steps 0 "$@" > "gpurun_out/envab_$name.log" 2>&1 \
      || { echo "$name failed"; tail -5 "gpurun_out/envab_$name.log"; exit 1; }
    echo "$name $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/envab_$name.log")"
  done
done
