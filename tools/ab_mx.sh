#!/bin/bash
# Interleaved A/B of two libfsdkr.so builds on the modexp shapes only (metric 2
# at 4 and 8 lanes, and the latency shapes with 896 instances, the GA chains of
# an 8-way shard rank, at 16/32/64 lanes).
# Usage (via gpurun): bash tools/ab_mx.sh TAG A.so B.so [rounds] [latency groups A] [latency groups B]
set -o pipefail
TAG=$1; A=$2; B=$3; ROUNDS=${4:-2}; LGA=${5:-16,32}; LGB=${6:-$LGA}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then export FSDKR_LIB=$A; LG=$LGA; else export FSDKR_LIB=$B; LG=$LGB; fi
    timeout -k 10 150 python tools/bench_modexp.py --count 65536 --reps 3 --widths 128,64 --groups 4,8 >> $O/mx_$v.jsonl 2>&1 || exit 1
    timeout -k 10 100 python tools/bench_modexp.py --count 896 --reps 3 --widths 128 --groups $LG >> $O/mxs_$v.jsonl 2>&1 || exit 1
    echo "round $r $v done"
  done
done
