#!/bin/bash
# Wave-per-instance fb_sched + vectorised recovery launch + SessionSet row gather:
# parity tests that cover them, the bench, configs[4] phases, an n = 64 trace.
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03z}
O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fixedbase or collect or configs or golden or reference or edge" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python $R/bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log > $O/bench.json
timeout -k 10 400 python $R/tools/phases_many.py --reps 3 > $O/phases.jsonl 2>&1 || { echo "phases failed"; tail -20 $O/phases.jsonl; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 $R/tools/prof_collect.py --full --steps 4 > $O/trace.log 2>&1) || { echo "trace failed"; tail -30 $O/trace.log; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python $R/tools/prof_summary.py "$f" --gap 10 --step 2 > $O/trace_summary.txt || exit 1
rm -rf $O/trace
timeout -k 10 300 python $R/tools/pack_many_cpu.py --split --reps 3 > $O/pack.jsonl 2>&1 || { echo "pack failed"; tail $O/pack.jsonl; exit 1; }

echo "all ok"
