#!/bin/bash
# dense-stage backward staging layout: kernel tests, bench x2, LDS-conflict PMC pass
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "dense_stage" -p no:cacheprovider > gpurun_out/r5/t_dsb.log 2>&1 || { tail -30 gpurun_out/r5/t_dsb.log; exit 1; }
tail -1 gpurun_out/r5/t_dsb.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/r5/b_dsb_$r.txt 2>&1 || exit 1
  tail -1 gpurun_out/r5/b_dsb_$r.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"])'
done
tools/pmc_session.sh dsb > gpurun_out/r5/pmc_dsb.log 2>&1 || { tail -5 gpurun_out/r5/pmc_dsb.log; exit 1; }
grep -E "dense_stage" gpurun_out/dsb_pmc.md
