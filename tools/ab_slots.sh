#!/bin/bash
# statistics-slot A/B (round 5): interleaved bench.py runs per model; results in gpurun_out/r5/
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
IDC_MICRO_GSUM_SLOTS=4 IDC_PHASES_DG_ONLY=1 timeout -k 10 120 ./conv_phases_x2 > gpurun_out/r5/conv_phases_dg_s4.txt 2>&1 || exit 1
run() {  # tag model env...
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --model $model --steps 30 --warmup 10 > gpurun_out/r5/b_$tag.txt 2>&1 || { tail -5 gpurun_out/r5/b_$tag.txt; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r5/b_$tag.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for r in 1 2; do
  run dn_base$r densenet121 IDC_STAT_SLOTS=0
  run dn_s4_$r densenet121 IDC_STAT_SLOTS=1 IDC_STAT_SLOTS_CAP=4
  run dn_s2_$r densenet121 IDC_STAT_SLOTS=1 IDC_STAT_SLOTS_CAP=2
  run dn_s8_$r densenet121 IDC_STAT_SLOTS=1 IDC_STAT_SLOTS_CAP=8
done
run mb_base mobilenetv2 IDC_STAT_SLOTS=0
run mb_s4 mobilenetv2 IDC_STAT_SLOTS=1 IDC_STAT_SLOTS_CAP=4
run vg_base vgg16 IDC_STAT_SLOTS=0
run vg_s4 vgg16 IDC_STAT_SLOTS=1 IDC_STAT_SLOTS_CAP=4
head -12 gpurun_out/r5/conv_phases_dg_s4.txt
