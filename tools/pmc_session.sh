#!/bin/bash
# usage: tools/pmc_session.sh <tag> [bench.py args...]
# One rocprofv3 PMC pass (8 SQ counters, kernel trace only) over a short bench run
# -> gpurun_out/<tag>_pmc.md (tools/pmc_summary.py: MFMA utilisation, LDS conflicts, waits)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/pmc
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAIT_ANY --kernel-trace --output-format csv \
  -d gpurun_out/pmc -o "$tag" -- python bench.py --steps 4 --warmup 3 --fit-steps 0 "$@" \
  > "gpurun_out/pmc_$tag.log" 2>&1 || exit $?
f=$(find gpurun_out/pmc -name "${tag}_counter_collection.csv" | head -1)
python tools/pmc_summary.py "${f%_counter_collection.csv}" --steps 3 --md "gpurun_out/${tag}_pmc.md" > /dev/null || exit $?
head -24 "gpurun_out/${tag}_pmc.md"
