#!/bin/bash
# Fresh-container HEAD check: full GPU suite, configs[4] phases, bench.
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03x; mkdir -p $O
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python $R/tools/phases_many.py --reps 3 > $O/phases.jsonl 2>&1 || { echo "phases failed"; tail -20 $O/phases.jsonl; exit 1; }
timeout -k 10 500 python $R/bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log > $O/bench.json
echo "all ok"
