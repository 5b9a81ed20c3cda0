#!/bin/bash
# n = 64 A/B: round-2 fb_sched (A) vs the ordered wave-per-instance one (C);
# fixed-base parity; configs[4] phases with C.
set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=12
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest $R/tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fixedbase or golden" > $R/gpurun_out/r03zb_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r03zb_tests.log; exit 1; }
tail -1 $R/gpurun_out/r03zb_tests.log
bash $R/tools/ab_n64.sh ab_fbsched2 abtmp/A.so abtmp/C.so 3 || { echo "ab failed"; exit 1; }
O=$R/gpurun_out/r03zb; mkdir -p $O
FSDKR_PREP_PROFILE=1 timeout -k 10 400 python $R/tools/phases_many.py --reps 3 > $O/phases.jsonl 2> $O/prep.txt || { echo "phases failed"; tail -20 $O/phases.jsonl; exit 1; }
echo "all ok"
