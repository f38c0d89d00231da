# round-6 GPU session (one call): mb_infer default cut 576 -- MobileNetV2 model tests, phase A/Bs,
# frozen-phase kernel trace
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_eval_gpu.py tests/test_fused_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "mobilenetv2" > gpurun_out/r6/t_mbmodel.log 2>&1 || { tail -40 gpurun_out/r6/t_mbmodel.log; exit 1; }
tail -2 gpurun_out/r6/t_mbmodel.log
tools/env_ab.sh 2 "fz|-" "fz0|IDC_MB_INFER=0" -- --model mobilenetv2 --phase frozen --steps 30 --warmup 10 || exit 1
tools/env_ab.sh 2 "ft|-" "ft0|IDC_MB_INFER=0" -- --model mobilenetv2 --phase finetune --steps 30 --warmup 10 || exit 1
tools/prof_session.sh mbv2_frozen_mbi --model mobilenetv2 --phase frozen || exit 1
