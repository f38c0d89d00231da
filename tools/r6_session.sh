# round-6 GPU session (one call): the whole-model gradient tests under the tightened fidelity bound
# (utils/fidelity.py: hard 2x, floor 0.02) with the margin report on
set -o pipefail
mkdir -p gpurun_out/r6
export IDC_FIDELITY_LOG=1
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_rccl_gpu.py -x -v -s --timeout 200 --timeout-method thread \
  > gpurun_out/r6/t_fid.log 2>&1 || { grep -E "fidelity|PASS|FAIL|Error" gpurun_out/r6/t_fid.log | tail -60; exit 1; }
grep -E "fidelity\]|passed|failed" gpurun_out/r6/t_fid.log | tail -60
