#!/bin/bash
# A/B a list of environment settings on the bench: tools/exp_env.sh "name|VAR=1 VAR2=x" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; envs="${spec#*|}"
  echo "== $name ($envs)"
  env $envs timeout -k 10 150 python bench.py --steps 100 --warmup 20 $BENCH_ARGS > gpurun_out/exp_$name.log 2>&1 || { tail -5 gpurun_out/exp_$name.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp_$name.log
done
