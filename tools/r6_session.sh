# round-6 GPU session (one call): stage-2 persistent backward kernel check, then an A/B of
# persistent launches on DenseNet-121 stage 2 (forward and backward)
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 240 --timeout-method thread \
  -k "dense_stage_bwd_matches_autograd and 256-6-128-12" > gpurun_out/r6/t_s2bwd.log 2>&1 || { tail -30 gpurun_out/r6/t_s2bwd.log; exit 1; }
tail -3 gpurun_out/r6/t_s2bwd.log
tools/env_ab.sh 2 "base|-" "b9216|IDC_DENSE_STAGE_BWD_MAXM=9216" "f9216|IDC_DENSE_STAGE_MAXM=9216" \
  "fb9216|IDC_DENSE_STAGE_MAXM=9216 IDC_DENSE_STAGE_BWD_MAXM=9216" || exit 1
