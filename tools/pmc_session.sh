#!/bin/bash
# usage: tools/pmc_session.sh <tag> [bench.py args...]
# Two rocprofv3 PMC passes (4 SQ counters each, --pmc only: no tracing domain beside it) over a
# short bench run with a shared tune cache, merged by tools/pmc_summary.py into
# gpurun_out/<tag>_pmc.md (MFMA utilisation, LDS bank conflicts, wave wait fraction, LDS stall).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/pmc
export IDC_TUNE_CACHE="$GRAFT_REPO_ROOT/gpurun_out/pmc/${tag}_tune.json"
rm -f "$IDC_TUNE_CACHE"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA \
  --output-format csv -d gpurun_out/pmc -o "${tag}_a" -- python bench.py --steps 4 --warmup 3 --fit-steps 0 "$@" \
  > "gpurun_out/pmc_${tag}_a.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_LDS \
  --output-format csv -d gpurun_out/pmc -o "${tag}_b" -- python bench.py --steps 4 --warmup 3 --fit-steps 0 "$@" \
  > "gpurun_out/pmc_${tag}_b.log" 2>&1 || exit $?
fa=$(find gpurun_out/pmc -name "${tag}_a_counter_collection.csv" | head -1)
fb=$(find gpurun_out/pmc -name "${tag}_b_counter_collection.csv" | head -1)
python tools/pmc_summary.py "${fa%_counter_collection.csv}" "${fb%_counter_collection.csv}" --steps 3 \
  --md "gpurun_out/${tag}_pmc.md" > /dev/null || exit $?
head -24 "gpurun_out/${tag}_pmc.md"
