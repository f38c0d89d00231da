#!/bin/bash
# round-5 closing measurements: profiles of the three models, phase benches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
IDC_PROF_GAPS=12 tools/prof_session.sh densenet121_bs256 > gpurun_out/r5/prof_dn_final.log 2>&1 || { tail -5 gpurun_out/r5/prof_dn_final.log; exit 1; }
IDC_PROF_GAPS=12 tools/prof_session.sh mobilenetv2_bs256 --model mobilenetv2 > gpurun_out/r5/prof_mb_final.log 2>&1 || { tail -5 gpurun_out/r5/prof_mb_final.log; exit 1; }
IDC_PROF_GAPS=12 tools/prof_session.sh vgg16_bs256 --model vgg16 > gpurun_out/r5/prof_vg_final.log 2>&1 || { tail -5 gpurun_out/r5/prof_vg_final.log; exit 1; }
for m in vgg16 mobilenetv2; do
  for ph in frozen finetune; do
    timeout -k 10 200 python bench.py --model $m --phase $ph --steps 30 --warmup 10 > gpurun_out/r5/b_ph_${m}_$ph.txt 2>&1 || { tail -5 gpurun_out/r5/b_ph_${m}_$ph.txt; exit 1; }
    echo "$m $ph $(tail -1 gpurun_out/r5/b_ph_${m}_$ph.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
head -5 gpurun_out/densenet121_bs256_timeline.txt gpurun_out/mobilenetv2_bs256_timeline.txt gpurun_out/vgg16_bs256_timeline.txt
