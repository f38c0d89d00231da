# round-6 GPU session (one call): one-pass depthwise backward -- kernel test, MobileNetV2 model
# tests with it on, A/B of the training step
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "dwconv" > gpurun_out/r6/t_dwf.log 2>&1 || { tail -40 gpurun_out/r6/t_dwf.log; exit 1; }
tail -2 gpurun_out/r6/t_dwf.log
IDC_DW_FUSED_BWD=1 timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "mobilenetv2" > gpurun_out/r6/t_dwf_model.log 2>&1 || { tail -40 gpurun_out/r6/t_dwf_model.log; exit 1; }
tail -2 gpurun_out/r6/t_dwf_model.log
tools/env_ab.sh 3 "sep|-" "fused|IDC_DW_FUSED_BWD=1" -- --model mobilenetv2 --steps 30 --warmup 10 || exit 1
