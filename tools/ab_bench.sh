#!/bin/bash
# Same-box A/B: the committed tree (ab_base/, built from `git archive HEAD`) vs the working tree,
# interleaved so box-to-box and drift effects cancel.  usage: tools/ab_bench.sh [rounds] [bench args]
mkdir -p gpurun_out
n=${1:-3}; shift
for i in $(seq "$n"); do
  for side in base new; do
    dir=.; [ "$side" = base ] && dir=ab_base
    (cd "$dir" && timeout -k 10 150 python bench.py --steps 100 --warmup 20 "$@") > "gpurun_out/ab_$side.log" 2>&1 \
      || { tail -5 "gpurun_out/ab_$side.log"; exit 1; }
    echo "$side $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/ab_$side.log")"
  done
done
