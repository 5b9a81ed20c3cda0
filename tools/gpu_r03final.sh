#!/bin/bash
# Round-3 final record at HEAD: the whole GPU suite, smoke(), the bench line (with
# the CPU baseline), a kernel-trace --stats profile of the bench command, and the
# configs[4] phases.
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03final}
O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 500 python $R/bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log > $O/bench.json
(cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1) || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/bench_kernel_stats.csv
grep '^{"metric"' $O/prof.log > $O/bench_under_rocprof.json
rm -rf $O/prof
timeout -k 10 400 python $R/tools/phases_many.py --reps 3 > $O/phases.jsonl 2>&1 || { echo "phases failed"; tail -20 $O/phases.jsonl; exit 1; }
echo "all ok"
