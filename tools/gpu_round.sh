#!/bin/bash
# One GPU-box session: GPU tests, the bench, a kernel-trace profile of the bench.
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh TAG [tests|bench|prof ...]
set -o pipefail
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# collect() runs 8 concurrent streams; rocprofv3's preload initialises HIP before
# bench.py can set this, so export it here (bench.py/conftest set it otherwise)
export GPU_MAX_HW_QUEUES=12
for step in "$@"; do
  case $step in
    tests) timeout -k 10 600 python -m pytest $R/tests -m gpu -x -q > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $OUT/tests.log; exit 1; } ;;
    bench) timeout -k 10 420 python $R/bench.py > $OUT/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $OUT/bench.log; exit 1; } ;;
    benchq) timeout -k 10 300 python $R/bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $OUT/bench.log; exit 1; } ;;
    prof) (cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1) || { echo "prof failed rc=$?"; tail -30 $OUT/prof.log; exit 1; } ;;
    trace) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o tr -- python3 $R/tools/prof_collect.py --full --steps 4 > $OUT/trace.log 2>&1) || { echo "trace failed rc=$?"; tail -30 $OUT/trace.log; exit 1; }
      f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
      python $R/tools/prof_summary.py "$f" --gap 10 --step 2 > $OUT/trace_summary.txt || exit 1 ;;
    *) timeout -k 10 420 bash -c "$step" > $OUT/extra.log 2>&1 || { echo "step failed rc=$?"; tail -30 $OUT/extra.log; exit 1; } ;;
  esac
  echo "step $step ok"
done
