# round-6 GPU session (one call): dense-stage kernel tests, row-resident stamps, same-box A/B
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "dense_stage" -p no:cacheprovider > gpurun_out/r6/t_ds.log 2>&1 || { tail -60 gpurun_out/r6/t_ds.log; exit 1; }
tail -1 gpurun_out/r6/t_ds.log
IDC_DS_ROWS=1 timeout -k 10 200 python -u tools/dense_stamps.py --md gpurun_out/r6/stamps_rows2.md > gpurun_out/r6/stamps_rows2.log 2>&1 || exit 1
IDC_DS_ROWS=1 IDC_DS_ROWS_RB=1 timeout -k 10 200 python -u tools/dense_stamps.py --md gpurun_out/r6/stamps_rows1.md > gpurun_out/r6/stamps_rows1.log 2>&1 || exit 1
tools/env_ab.sh 2 "rows2|IDC_DS_ROWS=1" "queue|IDC_DS_ROWS=0" "rows1|IDC_DS_ROWS=1 IDC_DS_ROWS_RB=1" || exit 1
