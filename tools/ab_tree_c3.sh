#!/bin/bash
# Interleaved A/B of two source trees on the configs[3] (n = 256) whole call.
# Usage (via gpurun): bash tools/ab_tree_c3.sh TAG treeA treeB [rounds]
set -o pipefail
TAG=$1; TA=$2; TB=$3; ROUNDS=${4:-2}
O=gpurun_out/$TAG; mkdir -p $O
export GPU_MAX_HW_QUEUES=12
for r in $(seq $ROUNDS); do
  for t in $TA $TB; do
    timeout -k 10 300 python $t/bench.py --steps 3 --warmup 1 --no-cpu-baseline --sessions 0 --config3-steps 3 \
      | sed "s|^|{\"tree\": \"$t\", \"r\": |; s|\$| }|" >> $O/bench.jsonl || exit 1
  done
  echo "round $r done"
done
