#!/bin/bash
# late round-5 env A/B on DenseNet-121 (interleaved, 2 rounds)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/r5/b_misc_$tag.txt 2>&1 || { tail -5 gpurun_out/r5/b_misc_$tag.txt; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r5/b_misc_$tag.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for r in 1 2; do
  run base$r IDC_X=0
  run wb2304_$r IDC_WG_BATCH_MAXM=2304
  run wb43k_$r IDC_WG_BATCH_MAXM=43264
  run dual$r IDC_DUAL_GRAPH=1
  run mainhi$r IDC_MAIN_PRIO=high
done
