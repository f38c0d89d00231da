#!/bin/bash
# stem pool (64-channel workgroups): tests, isolated kernel times, DenseNet bench x2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5 gpurun_out/pp2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pool" -p no:cacheprovider > gpurun_out/r5/t_pool2.log 2>&1 || { tail -30 gpurun_out/r5/t_pool2.log; exit 1; }
tail -1 gpurun_out/r5/t_pool2.log
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/pp2/img1 -o pool -- python3 tools/micro_pool.py > gpurun_out/r5/pool2_img1.log 2>&1 || exit 1
python -c "
import sqlite3,glob
c=sqlite3.connect(glob.glob('gpurun_out/pp2/img1/pool_results.db')[0])
for r in c.execute('select name, count(*), avg(end-start)/1000.0, min(end-start)/1000.0 from kernels group by name'):
    print(r[0][:50], r[1], 'avg %.1f us min %.1f us' % (r[2], r[3]))
"
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/r5/b_pool2_$r.txt 2>&1 || exit 1
  tail -1 gpurun_out/r5/b_pool2_$r.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"])'
done
