#!/bin/bash
# Interleaved A/B of two libfsdkr.so builds: bench.py's n = 256 whole call
# (configs[3]) and the n = 64 call.  Usage: bash tools/ab_n256.sh TAG A.so B.so [rounds]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; ROUNDS=${4:-2}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then export FSDKR_LIB=$A; else export FSDKR_LIB=$B; fi
    timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --sessions 0 --config3-steps 3 >> $O/bench_$v.jsonl 2>&1 || exit 1
    echo "round $r $v done"
  done
done
