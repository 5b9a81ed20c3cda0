#!/bin/bash
# round 6: emulated 8-way n = 64 rank at the r06m-record commit (15818d8, its own
# bench.py and package staged under abtmp/old) against HEAD, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zk_reg; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python $R/abtmp/old/bench.py --steps 10 --warmup 2 --emulate-shard 8 --no-cpu-baseline --sessions 0 \
    --config3-steps 0 >> $O/old.jsonl 2>> $O/old.err || { echo old failed; tail -5 $O/old.err; exit 1; }
  timeout -k 10 300 python $R/bench.py --steps 10 --warmup 2 --emulate-shard 8 --no-cpu-baseline --sessions 0 \
    --config3-steps 0 >> $O/head.jsonl 2>> $O/head.err || { echo head failed; tail -5 $O/head.err; exit 1; }
  echo "round $r done"
done
