#!/bin/bash
# round 6: bisect of the emulated 8-way n = 64 rank (21.8 ms at 15818d8, 25.2 at HEAD):
# 63fd1c8 and a35e3f6 (each its own bench.py and package under abtmp/old_*), HEAD, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zl_bis; mkdir -p $O
for r in 1 2; do
  for v in old_63fd1c8 old_a35e3f6 head; do
    B=$R/abtmp/$v/bench.py; [ $v = head ] && B=$R/bench.py
    timeout -k 10 300 python $B --steps 10 --warmup 2 --emulate-shard 8 --no-cpu-baseline --sessions 0 \
      --config3-steps 0 >> $O/$v.jsonl 2>> $O/$v.err || { echo $v failed; tail -5 $O/$v.err; exit 1; }
  done
  echo "round $r done"
done
