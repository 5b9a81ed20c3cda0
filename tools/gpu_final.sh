#!/bin/bash
# Round-end GPU session: parity tests, bench (with CPU baseline), kernel-trace
# profile of the bench, per-rank shard latency (emulated 2/4/8-way shards).
set -o pipefail
TAG=${1:-final}
bash tools/gpu_round.sh $TAG tests bench prof || exit 1
R=${GRAFT_REPO_ROOT:-$(pwd)}
python3 tools/prof_summary.py $(ls $R/gpurun_out/$TAG/prof/*kernel_trace.csv | head -1) > $R/gpurun_out/$TAG/prof_summary.txt || exit 1
for w in 2 4 8; do
  timeout -k 10 200 python bench.py --emulate-shard $w --steps 5 > $R/gpurun_out/$TAG/shard$w.log 2>&1 || { echo "shard $w failed"; exit 1; }
  tail -1 $R/gpurun_out/$TAG/shard$w.log
done
