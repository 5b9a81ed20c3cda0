#!/bin/bash
# Interleaved whole-call n = 64 bench over several libfsdkr.so builds (same Python).
# Usage (via gpurun): bash tools/ab_libs_n64.sh TAG "a.so b.so ..." [rounds]
set -o pipefail
TAG=$1; LIBS=$2; ROUNDS=${3:-3}
O=gpurun_out/$TAG; mkdir -p $O
export GPU_MAX_HW_QUEUES=12
for r in $(seq $ROUNDS); do
  for v in $LIBS; do
    FSDKR_LIB=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0 \
      | sed "s|^|{\"lib\": \"$v\", \"r\": |; s|\$| }|" >> $O/bench.jsonl || exit 1
  done
  echo "round $r done"
done
