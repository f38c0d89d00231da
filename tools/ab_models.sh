#!/bin/bash
# bench.py on every model, twice, interleaved (round 5); results in gpurun_out/r5/
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
tag=${1:-cur}
for r in 1 2; do
  for m in densenet121 mobilenetv2 vgg16; do
    timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5/b_${tag}_${m}_$r.txt 2>&1 || { tail -5 gpurun_out/r5/b_${tag}_${m}_$r.txt; exit 1; }
    echo "$tag $m $r $(tail -1 gpurun_out/r5/b_${tag}_${m}_$r.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
