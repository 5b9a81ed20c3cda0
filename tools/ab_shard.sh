#!/bin/bash
# Emulated shard ranks (bench.py --emulate-shard W, rank 0's whole call) for a
# set of library builds and GA CU-split sizes, interleaved.
# Usage (via gpurun): bash tools/ab_shard.sh TAG "W1 W2" "lib1:cus1 lib2:cus2 ..." [rounds]
set -o pipefail
TAG=$1; WS=$2; VARS=$3; ROUNDS=${4:-2}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for W in $WS; do
    for v in $VARS; do
      lib=${v%%:*}; cus=${v##*:}
      FSDKR_LIB=$lib FSDKR_SHARD_GA_CUS=$cus timeout -k 10 200 python bench.py --steps 10 --warmup 2 --emulate-shard $W \
        | sed "s|^|{\"lib\": \"$lib\", \"cus\": $cus, \"W\": $W, \"r\": |; s|\$| }|" >> $O/shard.jsonl 2>> $O/shard.err || exit 1
    done
  done
  echo "round $r done"
done
