# round-6 GPU session (one call): kernel tests of the dense-stage launches, the fused DP test, and
# a same-box A/B of the row-resident dense stage (tools/env_ab.sh)
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "dense_stage" -p no:cacheprovider > gpurun_out/r6/t_ds.log 2>&1 || { tail -60 gpurun_out/r6/t_ds.log; exit 1; }
tail -1 gpurun_out/r6/t_ds.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_dp_gpu.py -p no:cacheprovider > gpurun_out/r6/t_dp.log 2>&1; grep DPCASE gpurun_out/dp_worker.log | cut -c1-300
tools/env_ab.sh 2 "rows2|IDC_DS_ROWS=1" "queue|IDC_DS_ROWS=0" "rows1|IDC_DS_ROWS=1 IDC_DS_ROWS_RB=1" || exit 1
