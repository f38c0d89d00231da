# round-6 GPU session (one call): fused MobileNetV2 inference block -- kernel tests, model-level
# inference / frozen-phase tests, then an A/B of the frozen-base phase and its kernel trace
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k mb_infer > gpurun_out/r6/t_mbi.log 2>&1 || { tail -40 gpurun_out/r6/t_mbi.log; exit 1; }
tail -3 gpurun_out/r6/t_mbi.log
timeout -k 10 400 python -u -m pytest tests/test_eval_gpu.py tests/test_fused_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "mobilenetv2" > gpurun_out/r6/t_mbmodel.log 2>&1 || { tail -40 gpurun_out/r6/t_mbmodel.log; exit 1; }
tail -3 gpurun_out/r6/t_mbmodel.log
tools/env_ab.sh 2 "mbi|-" "mbi0|IDC_MB_INFER=0" -- --model mobilenetv2 --phase frozen --steps 30 --warmup 10 || exit 1
tools/prof_session.sh mbv2_frozen_mbi --model mobilenetv2 --phase frozen || exit 1
