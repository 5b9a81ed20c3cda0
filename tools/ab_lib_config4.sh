#!/bin/bash
# Interleaved A/B of two builds of libfsdkr.so on configs[4] (1024 sessions,
# bench.py's collect_many step) and the n = 64 headline of the same run.
# Usage (via gpurun): bash tools/ab_lib_config4.sh TAG path/to/A.so path/to/B.so [rounds]
set -o pipefail
TAG=$1; A=$2; B=$3; ROUNDS=${4:-2}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then export FSDKR_LIB=$A; else export FSDKR_LIB=$B; fi
    timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --config3-steps 0 --session-steps 3 \
      >> $O/bench_$v.jsonl 2>> $O/bench_$v.err || exit 1
    echo "round $r $v done"
  done
done
