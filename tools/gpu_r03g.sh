#!/bin/bash
# One GPU call: parity tests of the changed kernels, collect A/B, shard split
# sweep, configs[4] phases (round 3).
set -o pipefail
export GPU_MAX_HW_QUEUES=12
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_modexp_gpu.py tests/test_fixedbase_gpu.py tests/test_collect_gpu.py tests/test_shard_batch.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
echo "tests ok"; tail -1 $O/tests.log
bash tools/ab_lib.sh r03g_ab abtmp/A.so abtmp/B2.so 1 || exit 1
bash tools/ab_shard.sh r03g_sh "8 4" "abtmp/B2.so:160 abtmp/B2.so:0 abtmp/B2.so:224" 1 || exit 1
timeout -k 10 300 python tools/phases_many.py --sessions 1024 --reps 2 > $O/phases_many.jsonl 2>&1 || { echo "phases failed"; tail -20 $O/phases_many.jsonl; exit 1; }
echo "all ok"
