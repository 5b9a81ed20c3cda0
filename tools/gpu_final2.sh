#!/bin/bash
# Round-end GPU session: parity tests, smoke, bench (with CPU baseline), a
# kernel-trace profile of whole collect() calls (the timed step), per-rank
# latency of emulated 2/4/8-way shards.  Usage: bash tools/gpu_final2.sh TAG
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
bash tools/gpu_round.sh $TAG tests bench || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
(cd /tmp && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=12 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o full -- python3 $R/tools/prof_collect.py --full --steps 4 > $O/prof.log 2>&1) || { echo prof failed; tail -20 $O/prof.log; exit 1; }
python3 tools/prof_summary.py --gap 10 --step -2 $(ls $O/prof/*kernel_trace.csv | head -1) > $O/prof_summary.txt || exit 1
echo prof ok
for w in 2 4 8; do
  timeout -k 10 200 python bench.py --emulate-shard $w --steps 6 --warmup 2 > $O/shard$w.log 2>&1 || { echo "shard $w failed"; exit 1; }
  tail -1 $O/shard$w.log
done
