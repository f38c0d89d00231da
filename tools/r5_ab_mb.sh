#!/bin/bash
# MobileNetV2 statistics-slot cap A/B (interleaved, 2 rounds)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --model mobilenetv2 --steps 30 --warmup 10 > gpurun_out/r5/b_mbcap_$tag.txt 2>&1 || { tail -5 gpurun_out/r5/b_mbcap_$tag.txt; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r5/b_mbcap_$tag.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for r in 1 2; do
  run c4_$r IDC_STAT_SLOTS_CAP=4
  run c2_$r IDC_STAT_SLOTS_CAP=2
  run c8_$r IDC_STAT_SLOTS_CAP=8
  run c16_$r IDC_STAT_SLOTS_CAP=16
done
