#!/bin/bash
# Interleaved A/B/C... of several builds of libfsdkr.so running one command on one
# box (same inputs); each variant's stdout is appended to out_<k>.jsonl.
# Usage (via gpurun): bash tools/ab_libs.sh TAG ROUNDS "python bench.py ..." lib0.so lib1.so ...
set -o pipefail
TAG=$1; ROUNDS=$2; CMD=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  k=0
  for lib in "$@"; do
    echo "$lib" > $O/lib_$k.txt
    FSDKR_LIB=$lib timeout -k 10 400 $CMD >> $O/out_$k.jsonl 2>> $O/err_$k.log \
      || { echo "variant $k ($lib) failed"; tail -5 $O/err_$k.log; exit 1; }
    echo "round $r variant $k done"
    k=$((k + 1))
  done
done
