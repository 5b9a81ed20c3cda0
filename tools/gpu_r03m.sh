#!/bin/bash
# Kernel-trace timelines of the emulated 8-way rank-0 whole call (GA CU split 160 and none).
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03m; mkdir -p $O
for cus in 160 0; do
  (cd /tmp && FSDKR_SHARD_GA_CUS=$cus timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$cus -o tr -- python3 $R/bench.py --emulate-shard 8 --steps 4 --warmup 2 --gap-ms 20 > $O/tr$cus.log 2>&1) || { echo "tr failed"; tail -20 $O/tr$cus.log; exit 1; }
  f=$(find $O/tr$cus -name "*kernel_trace.csv" | head -1)
  python $R/tools/prof_summary.py "$f" --gap 10 --step -2 > $O/tr${cus}_summary.txt || exit 1
  rm -rf $O/tr$cus
done
echo "all ok"
