#!/bin/bash
# r04b: full GPU suite on the quotient-scaled build, then QS on/off A/B of the
# latency modexp shapes and the n = 64 whole call
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
export GPU_MAX_HW_QUEUES=12
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for q in 0 1; do
    FSDKR_QS=$q timeout -k 10 150 python tools/bench_modexp.py --count 7680 --reps 3 --widths 128,64 --groups 8,16 >> $O/mxs_qs$q.jsonl 2>> $O/mx.err || exit 1
  done
done
bash tools/ab_env.sh r04b 3 "--steps 10 --warmup 2" "FSDKR_QS=0" "FSDKR_QS=1" || exit 1
