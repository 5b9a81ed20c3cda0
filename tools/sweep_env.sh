#!/bin/bash
# Tuning-knob sweep of the n = 64 collect bench.  Each argument is a "+"-separated
# list of VAR=VALUE settings for one bench run ("-" = defaults).
# Usage (via gpurun): bash tools/sweep_env.sh TAG FSDKR_GA_FIRST=7 FSDKR_RESERVE_CUS=16+FSDKR_RESERVE_EXCL=0 ...
set -o pipefail
TAG=${1:-sweep}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=12
i=0
for a in "$@"; do
  i=$((i+1))
  envs=(); [[ $a != - ]] && IFS=+ read -ra envs <<< "$a"
  env "${envs[@]}" timeout -k 10 300 python $R/bench.py --no-cpu-baseline --steps 5 $BENCH_ARGS > $OUT/bench_$i.log 2>&1 || { echo "bench $a failed rc=$?"; tail -30 $OUT/bench_$i.log; exit 1; }
  echo "$a $(tail -1 $OUT/bench_$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
