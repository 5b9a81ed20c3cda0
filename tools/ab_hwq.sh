#!/bin/bash
# collect() knob A/B at shard 1 and 8 under 8 and 12 hardware queues (via gpurun).
set -o pipefail
O=gpurun_out/${1:-hwq}; shift; mkdir -p $O
for q in 8 12; do
  for w in 8 1; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python tools/ab_collect.py --shard $w --rounds 4 "$@" > $O/q${q}_w$w.log 2>&1 || exit 1
    grep -o '"config": "[^"]*"\|"median_ms": [0-9.]*' $O/q${q}_w$w.log | paste - - | sed "s/^/q=$q w=$w /"
  done
done
