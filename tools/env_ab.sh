#!/bin/bash
# The one same-box A/B harness: bench.py under several environment settings (and/or models),
# interleaved round by round so box drift cancels.  One line per run: name, ms/step, value.
#
# usage: tools/env_ab.sh ROUNDS "NAME|ENV..." ["NAME|ENV..." ...] [-- bench.py args]
#   NAME   a label (also the log name: gpurun_out/ab/NAME_ROUND.log)
#   ENV    space-separated VAR=value settings for that run ("-" for none); a MODEL=x entry becomes
#          `--model x` for that run only
# Defaults: --steps 30 --warmup 10 (override after --).  Every run is under its own time limit and
# the harness stops at the first failure (no retries on the GPU).
#
# Recipes of the round-5 experiments this replaces (BASELINE.md round-5 notes):
#   dense-stage grid        tools/env_ab.sh 2 "base|-" "g512|IDC_DS_GRID=512" "g384|IDC_DS_GRID=384" "g192|IDC_DS_GRID=192"
#   persistent stage cuts   tools/env_ab.sh 2 "base|-" "bwd2304|IDC_DENSE_STAGE_BWD_MAXM=2304" "fwd256|IDC_DENSE_STAGE_MAXM=256"
#   statistics slot caps    tools/env_ab.sh 2 "s1|IDC_STAT_SLOTS=0" "s4|IDC_STAT_SLOTS_CAP=4" "s8|IDC_STAT_SLOTS_CAP=8"
#   same, MobileNetV2       tools/env_ab.sh 2 "s1|MODEL=mobilenetv2 IDC_STAT_SLOTS=0" "s4|MODEL=mobilenetv2"
#   pool kernels            tools/env_ab.sh 2 "img1|IDC_POOL_IMG=1" "img0|IDC_POOL_IMG=0"
#   side-lane flush         tools/env_ab.sh 2 "f2|IDC_SIDE_FLUSH=2" "f4|IDC_SIDE_FLUSH=4" "f8|IDC_SIDE_FLUSH=8"
#   all three models        tools/env_ab.sh 2 "dn|MODEL=densenet121" "mb|MODEL=mobilenetv2" "vg|MODEL=vgg16"
#   phases                  tools/env_ab.sh 1 "vgf|MODEL=vgg16" -- --phase frozen --steps 30 --warmup 10
# Tree-vs-tree A/B (committed HEAD against the working tree): tools/ab_bench.sh.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out/ab
n=$1; shift
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" = "--" ] && shift
args=("$@"); [ ${#args[@]} -eq 0 ] && args=(--steps 30 --warmup 10)
for i in $(seq "$n"); do
  for spec in "${specs[@]}"; do
    name="${spec%%|*}"; envs="${spec#*|}"; [ "$envs" = "-" ] && envs=""
    model=(); keep=()
    for e in $envs; do
      case "$e" in MODEL=*) model=(--model "${e#MODEL=}");; *) keep+=("$e");; esac
    done
    log="gpurun_out/ab/${name}_$i.log"
    env "${keep[@]}" timeout -k 10 200 python bench.py "${model[@]}" "${args[@]}" > "$log" 2>&1 \
      || { echo "$name failed"; tail -5 "$log"; exit 1; }
    echo "$name $i $(tail -1 "$log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
