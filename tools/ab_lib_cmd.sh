#!/bin/bash
# Interleaved A/B of two builds of libfsdkr.so running one command (its stdout
# appended per variant).  Usage (via gpurun):
#   bash tools/ab_lib_cmd.sh TAG A.so B.so ROUNDS "python bench.py ..."
set -o pipefail
TAG=$1; A=$2; B=$3; ROUNDS=$4; CMD=$5
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for v in A B; do
    if [ $v = A ]; then export FSDKR_LIB=$A; else export FSDKR_LIB=$B; fi
    timeout -k 10 400 $CMD >> $O/out_$v.jsonl 2>> $O/err_$v.log || { echo "variant $v failed"; tail -5 $O/err_$v.log; exit 1; }
    echo "round $r $v done"
  done
done
