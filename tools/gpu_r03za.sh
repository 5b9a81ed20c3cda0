#!/bin/bash
# n = 64 A/B of the round-2 fb_sched (A) vs the wave-per-instance one (B), then
# the configs[4] phases with the prepare breakdown (FSDKR_PREP_PROFILE) at HEAD.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
export GPU_MAX_HW_QUEUES=12
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread -k "collect or recover or configs or reference" > $R/gpurun_out/r03za_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/r03za_tests.log; exit 1; }
tail -2 $R/gpurun_out/r03za_tests.log
bash $R/tools/ab_n64.sh ab_fbsched abtmp/A.so abtmp/B.so 3 || { echo "ab failed"; exit 1; }
O=$R/gpurun_out/r03za; mkdir -p $O
FSDKR_PREP_PROFILE=1 timeout -k 10 400 python $R/tools/phases_many.py --reps 3 > $O/phases.jsonl 2> $O/prep.txt || { echo "phases failed"; tail -20 $O/prep.txt; exit 1; }
echo "all ok"
