#!/bin/bash
# usage: tools/prof_session.sh <tag> [bench.py args...]   (env vars pass through)
# rocprofv3 kernel trace of a short bench run -> gpurun_out/<tag>_kernels.md (per-step summary)
# and gpurun_out/<tag>_timeline.txt (critical-path view of one step)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/prof
timeout -k 10 240 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/prof -o "$tag" -- \
  python bench.py --steps 10 --warmup 5 --fit-steps 0 "$@" > "gpurun_out/prof_$tag.log" 2>&1 || exit $?
db=$(find gpurun_out/prof -name "${tag}_results.db" | head -1)
python tools/prof_summary.py "$db" --steps 10 --md "gpurun_out/${tag}_kernels.md" > /dev/null || exit $?
python tools/timeline.py "$db" --top 14 --gaps ${IDC_PROF_GAPS:-0} > "gpurun_out/${tag}_timeline.txt" || exit $?
head -8 "gpurun_out/${tag}_kernels.md"
head -7 "gpurun_out/${tag}_timeline.txt"
