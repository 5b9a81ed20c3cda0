#!/bin/bash
# Interleaved A/B of two builds of libfsdkr.so on one GPU box (same inputs, same
# box): the modexp shapes (metric 2 and the latency shapes) and bench.py's whole
# collect() step at n = 64 and an emulated 8-way shard rank.
# Usage (via gpurun): bash tools/ab_lib.sh TAG path/to/A.so path/to/B.so [rounds]
set -o pipefail
TAG=$1; A=$2; B=$3; ROUNDS=${4:-2}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then export FSDKR_LIB=$A; else export FSDKR_LIB=$B; fi
    timeout -k 10 150 python tools/bench_modexp.py --count 65536 --reps 3 --widths 128,64 --groups 4,8 >> $O/mx_$v.jsonl 2>&1 || exit 1
    timeout -k 10 100 python tools/bench_modexp.py --count 7680 --reps 3 --widths 128,64 --groups 8,16 >> $O/mxs_$v.jsonl 2>&1 || exit 1
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0 >> $O/bench_$v.jsonl 2>&1 || exit 1
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --emulate-shard 8 >> $O/shard8_$v.jsonl 2>&1 || exit 1
    echo "round $r $v done"
  done
done
