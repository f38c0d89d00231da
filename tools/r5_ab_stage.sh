#!/bin/bash
# persistent-stage A/B after the round-5 kernel changes (interleaved, 2 rounds)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/r5/b_st_$tag.txt 2>&1 || { tail -5 gpurun_out/r5/b_st_$tag.txt; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r5/b_st_$tag.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for r in 1 2; do
  run base$r IDC_X=0
  run bwd2304_$r IDC_DENSE_STAGE_BWD_MAXM=2304
  run fwd256_$r IDC_DENSE_STAGE_MAXM=256
  run both_$r IDC_DENSE_STAGE_BWD_MAXM=2304 IDC_DENSE_STAGE_MAXM=256
done
