#!/bin/bash
# Kernel-trace timelines: the emulated 8-way rank-0 whole call and the n = 64 whole call.
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03h; mkdir -p $O
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr8 -o tr -- python3 $R/bench.py --emulate-shard 8 --steps 4 --warmup 2 --gap-ms 20 > $O/tr8.log 2>&1) || { echo "tr8 failed"; tail -20 $O/tr8.log; exit 1; }
f=$(find $O/tr8 -name "*kernel_trace.csv" | head -1)
python $R/tools/prof_summary.py "$f" --gap 10 --step -2 > $O/tr8_summary.txt || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr64 -o tr -- python3 $R/tools/prof_collect.py --full --steps 4 > $O/tr64.log 2>&1) || { echo "tr64 failed"; tail -20 $O/tr64.log; exit 1; }
f=$(find $O/tr64 -name "*kernel_trace.csv" | head -1)
python $R/tools/prof_summary.py "$f" --gap 10 --step -2 > $O/tr64_summary.txt || exit 1
rm -rf $O/tr8 $O/tr64
echo "all ok"
