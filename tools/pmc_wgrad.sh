cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmcw
CFG="b3c2:1:14,b3c2:0:32,b4c2:5:4,b4c2:1:4,b2c2:7:104"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAIT_ANY --output-format csv -d gpurun_out/pmcw -o p1 -- python tools/bench_wgrad.py --only $CFG --iters 6 > gpurun_out/pmcw/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmcw -o p2 -- python tools/bench_wgrad.py --only $CFG --iters 6 > gpurun_out/pmcw/p2.log 2>&1 || exit 1
f1=$(find gpurun_out/pmcw -name "p1_counter_collection.csv" | head -1); f2=$(find gpurun_out/pmcw -name "p2_counter_collection.csv" | head -1)
python tools/pmc_kernels.py "${f1%_counter_collection.csv}" --skip 0
python tools/pmc_kernels.py "${f2%_counter_collection.csv}" --skip 0
