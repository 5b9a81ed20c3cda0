#!/bin/bash
# Full GPU suite at HEAD, then the early share-recovery launch A/B (shard ranks, n = 64 whole call).
set -o pipefail
export GPU_MAX_HW_QUEUES=12
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests ok"; tail -1 $O/tests.log
bash tools/ab_shard.sh r03j_sh "8 4" "abtmp/B3.so:160 fs-dkr_amd/fsdkr/libfsdkr.so:160" 2 || exit 1
for r in 1 2; do
  for v in abtmp/B3.so fs-dkr_amd/fsdkr/libfsdkr.so; do
    FSDKR_LIB=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0 | sed "s|^|{\"lib\": \"$v\", \"r\": |; s|\$| }|" >> $O/bench.jsonl || exit 1
  done
done
echo "all ok"
