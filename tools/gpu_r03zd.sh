#!/bin/bash
# Correct-key prestart (configs[4]): parity tests over the multi-session and
# single-call paths, configs[4] phases, the bench line.
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03zd; mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread -k "configs or collect or golden or edge or shard or reference" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python $R/tools/phases_many.py --reps 3 > $O/phases.jsonl 2>&1 || { echo "phases failed"; tail -20 $O/phases.jsonl; exit 1; }
timeout -k 10 500 python $R/bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log > $O/bench.json
echo "all ok"
