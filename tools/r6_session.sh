# round-6 GPU session (one call): per-image TRAINING launch of DenseNet stages 1-2
# (dense_infer.hip dense_img_fwd) -- kernel tests, DenseNet model tests, full-step A/B, trace
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "persistent_matches_reference" > gpurun_out/r6/t_img.log 2>&1 || { tail -40 gpurun_out/r6/t_img.log; exit 1; }
tail -2 gpurun_out/r6/t_img.log
timeout -k 10 400 python -u -m pytest tests/test_eval_gpu.py tests/test_fused_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "densenet or dense_stage or dense_img" > gpurun_out/r6/t_img_model.log 2>&1 || { tail -40 gpurun_out/r6/t_img_model.log; exit 1; }
tail -2 gpurun_out/r6/t_img_model.log
tools/env_ab.sh 2 "img|-" "img0|IDC_DENSE_IMG=0" || exit 1
tools/prof_session.sh dn121_img || exit 1
