#!/bin/bash
# MobileNetV2 depthwise BN backward staged by its consumers (IDC_MBV2_DW_AFF=1) vs materialised
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --model mobilenetv2 --steps 30 --warmup 10 > gpurun_out/r5/b_dwaff_$tag.txt 2>&1 || { tail -5 gpurun_out/r5/b_dwaff_$tag.txt; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r5/b_dwaff_$tag.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for r in 1 2; do
  run base$r IDC_X=0
  run aff$r IDC_MBV2_DW_AFF=1
done
