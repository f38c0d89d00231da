#!/bin/bash
# pool-kernel A/B (round 5): tests, then bench.py under each variant; results in gpurun_out/r5/
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
timeout -k 10 120 ./conv_phases_x > gpurun_out/r5/conv_phases_dg.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pool" > gpurun_out/r5/t_pool.log 2>&1 || { tail -30 gpurun_out/r5/t_pool.log; exit 1; }
tail -1 gpurun_out/r5/t_pool.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 10 ${BENCH_ARGS} > gpurun_out/r5/b_$tag.txt 2>&1 || { tail -5 gpurun_out/r5/b_$tag.txt; exit 1; }
  echo "$tag $(tail -1 gpurun_out/r5/b_$tag.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
run dn_img1 IDC_POOL_IMG=1
run dn_img0 IDC_POOL_IMG=0
run dn_img1b IDC_POOL_IMG=1
run dn_div2 IDC_POOL_GRID_DIV=2
run dn_sl4 IDC_STAT_SLOTS=1 IDC_STAT_SLOTS_CAP=4
run dn_sl16 IDC_STAT_SLOTS=1
run dn_img1c IDC_POOL_IMG=1
BENCH_ARGS="--model vgg16" run vg_img1 IDC_POOL_IMG=1
BENCH_ARGS="--model vgg16" run vg_img0 IDC_POOL_IMG=0
head -30 gpurun_out/r5/conv_phases_dg.txt
