#!/bin/bash
# Interleaved A/B of two source trees (each with its own bench.py, fsdkr package
# and libfsdkr.so): n = 64 whole-call bench and emulated shard ranks.
# Usage (via gpurun): bash tools/ab_tree.sh TAG treeA treeB [rounds] ["W1 W2"]
set -o pipefail
TAG=$1; TA=$2; TB=$3; ROUNDS=${4:-2}; WS=${5:-"8 4"}
O=gpurun_out/$TAG; mkdir -p $O
export GPU_MAX_HW_QUEUES=12
for r in $(seq $ROUNDS); do
  for t in $TA $TB; do
    timeout -k 10 200 python $t/bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0 \
      | sed "s|^|{\"tree\": \"$t\", \"r\": |; s|\$| }|" >> $O/bench.jsonl || exit 1
    for W in $WS; do
      timeout -k 10 200 python $t/bench.py --steps 10 --warmup 2 --emulate-shard $W \
        | sed "s|^|{\"tree\": \"$t\", \"W\": $W, \"r\": |; s|\$| }|" >> $O/shard.jsonl || exit 1
    done
  done
  echo "round $r done"
done
