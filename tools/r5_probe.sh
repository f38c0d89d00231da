#!/bin/bash
# round-5 probe: concat-gradient dgrad micro (4 slot copies), DenseNet profile, stem-pool kernels
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5 gpurun_out/pp
IDC_MICRO_GSUM_SLOTS=4 IDC_PHASES_DG_ONLY=1 timeout -k 10 120 ./conv_phases_x2 > gpurun_out/r5/micro_vf.txt 2>&1 || exit 1
grep -E "back-to-back|span|eligible" gpurun_out/r5/micro_vf.txt
IDC_PROF_GAPS=12 tools/prof_session.sh dn_vf > gpurun_out/r5/prof_dn_vf.log 2>&1 || { tail -5 gpurun_out/r5/prof_dn_vf.log; exit 1; }
for v in 1 0; do
  IDC_POOL_IMG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pp/img$v -o pool -- python3 tools/micro_pool.py > gpurun_out/r5/pool_img$v.log 2>&1 || exit 1
done
find gpurun_out/pp -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -8; done
