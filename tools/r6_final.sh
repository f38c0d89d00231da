# round-6 closing GPU session (one call): the whole GPU suite, smoke(), and the 1-GPU bench at HEAD
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r6/final_suite.log 2>&1 || { tail -40 gpurun_out/r6/final_suite.log; exit 1; }
tail -3 gpurun_out/r6/final_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6/final_smoke.log 2>&1 \
  || { tail -20 gpurun_out/r6/final_smoke.log; exit 1; }
tail -1 gpurun_out/r6/final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r6/final_bench.log 2>&1 || { tail -20 gpurun_out/r6/final_bench.log; exit 1; }
tail -1 gpurun_out/r6/final_bench.log
