# round-6 GPU session (one call): same-box A/B of the row-resident stage-3 forward
set -o pipefail
mkdir -p gpurun_out/r6
tools/env_ab.sh 3 "base|-" "rows3|IDC_DS_ROWS=1 IDC_DS_ROWS_RB=1" "rows3rb2|IDC_DS_ROWS=1 IDC_DS_ROWS_RB=2" || exit 1
