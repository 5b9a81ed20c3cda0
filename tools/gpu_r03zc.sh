#!/bin/bash
# Whole-call kernel timelines at n = 64 for three fb_sched builds (A: round 2,
# C: wave per instance at priority 3, D: the same without the priority raise),
# then an interleaved A / D bench A/B.
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03zc; mkdir -p $O
for v in A C D; do
  (cd /tmp && FSDKR_LIB=$R/abtmp/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$v -o tr -- python3 $R/tools/prof_collect.py --full --steps 4 > $O/tr$v.log 2>&1) || { echo "trace $v failed"; tail -20 $O/tr$v.log; exit 1; }
  f=$(find $O/tr$v -name "*kernel_trace.csv" | head -1)
  python $R/tools/prof_summary.py "$f" --gap 10 --step -2 > $O/tr${v}_summary.txt || exit 1
  python $R/tools/prof_summary.py "$f" --gap 10 --step -3 > $O/tr${v}_summary3.txt || exit 1
  rm -rf $O/tr$v
done
bash $R/tools/ab_n64.sh ab_fbsched3 abtmp/A.so abtmp/D.so 2 || { echo "ab failed"; exit 1; }
echo "all ok"
