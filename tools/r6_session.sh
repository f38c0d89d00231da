# round-6 GPU session (one call): whole dense blocks in inference mode (dense_infer.hip) -- kernel
# test, DenseNet model tests, frozen-phase A/B of the late stages, frozen-phase traces
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "dense_infer" > gpurun_out/r6/t_di.log 2>&1 || { tail -40 gpurun_out/r6/t_di.log; exit 1; }
tail -2 gpurun_out/r6/t_di.log
timeout -k 10 400 python -u -m pytest tests/test_eval_gpu.py tests/test_fused_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "densenet" > gpurun_out/r6/t_di_model.log 2>&1 || { tail -40 gpurun_out/r6/t_di_model.log; exit 1; }
tail -2 gpurun_out/r6/t_di_model.log
tools/env_ab.sh 2 "e0|-" "late|IDC_DENSE_INFER_LATE=1" "r4|IDC_DENSE_INFER_LATE=1 IDC_DENSE_INFER_ROWS=4" \
  -- --phase frozen --steps 30 --warmup 10 || exit 1
tools/prof_session.sh dn121_frozen_e0 --phase frozen || exit 1
IDC_DENSE_INFER_LATE=1 tools/prof_session.sh dn121_frozen_late --phase frozen || exit 1
