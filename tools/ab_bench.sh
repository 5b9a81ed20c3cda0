#!/bin/bash
# Interleaved A/B of two libfsdkr.so builds on bench.py's n = 64 whole-call step
# (same box, alternating A B A B ...).  Usage: bash tools/ab_bench.sh TAG A.so B.so [rounds] [extra bench args]
set -o pipefail
TAG=$1; A=$2; B=$3; ROUNDS=${4:-3}; shift 4; EXTRA="$@"
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then export FSDKR_LIB=$A; else export FSDKR_LIB=$B; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --sessions 0 --config3-steps 0 $EXTRA >> $O/bench_$v.jsonl 2>&1 || exit 1
    echo "round $r $v done"
  done
done
