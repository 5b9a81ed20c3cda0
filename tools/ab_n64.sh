#!/bin/bash
# Interleaved A/B of two libfsdkr.so builds on one box: bench.py's whole n = 64
# collect() step only.  Usage (via gpurun): bash tools/ab_n64.sh TAG A.so B.so [rounds]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; ROUNDS=${4:-3}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then export FSDKR_LIB=$A; else export FSDKR_LIB=$B; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0 >> $O/bench_$v.jsonl 2>&1 || exit 1
    echo "round $r $v done"
  done
done
