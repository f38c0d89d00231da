#!/bin/bash
# usage: tools/pmc_bytes.sh <tag> [bench.py args...]
# Two rocprofv3 PMC passes for HBM traffic (FETCH_SIZE, then WRITE_SIZE: 3 + 2 TCC counters do not
# fit one pass) over a short bench run, merged by tools/pmc_summary.py --bytes into
# gpurun_out/<tag>_bytes.md (per-kernel bytes read / written and the implied bandwidth).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/pmc
export IDC_TUNE_CACHE="$GRAFT_REPO_ROOT/gpurun_out/pmc/${tag}_tune.json"
rm -f "$IDC_TUNE_CACHE"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc -o "${tag}_c" -- python bench.py --steps 4 --warmup 3 --fit-steps 0 "$@" \
  > "gpurun_out/pmc_${tag}_c.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE \
  --output-format csv -d gpurun_out/pmc -o "${tag}_d" -- python bench.py --steps 4 --warmup 3 --fit-steps 0 "$@" \
  > "gpurun_out/pmc_${tag}_d.log" 2>&1 || exit $?
fc=$(find gpurun_out/pmc -name "${tag}_c_counter_collection.csv" | head -1)
fd=$(find gpurun_out/pmc -name "${tag}_d_counter_collection.csv" | head -1)
python tools/pmc_summary.py "${fc%_counter_collection.csv}" "${fd%_counter_collection.csv}" --steps 3 --bytes \
  --md "gpurun_out/${tag}_bytes.md" > /dev/null || exit $?
head -30 "gpurun_out/${tag}_bytes.md"
