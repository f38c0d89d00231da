# closing GPU session (one gpurun call): the whole GPU suite, smoke() and the 1-GPU bench at HEAD
#   gpurun --timeout 1200 -- "bash tools/gpu_closing.sh"   (logs under gpurun_out/closing/)
set -o pipefail
mkdir -p gpurun_out/closing
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/closing/suite.log 2>&1 || { tail -40 gpurun_out/closing/suite.log; exit 1; }
tail -3 gpurun_out/closing/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/closing/smoke.log 2>&1 \
  || { tail -20 gpurun_out/closing/smoke.log; exit 1; }
tail -1 gpurun_out/closing/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/closing/bench.log 2>&1 || { tail -20 gpurun_out/closing/bench.log; exit 1; }
tail -1 gpurun_out/closing/bench.log
