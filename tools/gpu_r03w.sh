#!/bin/bash
# configs[4] phases in collect_many's order, and a kernel trace of the same calls.
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03w; mkdir -p $O
timeout -k 10 400 python $R/tools/phases_many.py --reps 3 > $O/phases.jsonl 2>&1 || { echo "phases failed"; tail -20 $O/phases.jsonl; exit 1; }
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr -- python3 $R/tools/phases_many.py --reps 2 --gap-ms 60 > $O/tr.log 2>&1) || { echo "trace failed"; tail -20 $O/tr.log; exit 1; }
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
for st in -2 -3 -4 -5; do python $R/tools/prof_summary.py "$f" --gap 40 --step $st > $O/tr_summary$st.txt || exit 1; done
rm -rf $O/tr
echo "all ok"
