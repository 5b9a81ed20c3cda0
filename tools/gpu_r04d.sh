#!/bin/bash
# r04d: GPU tests touched this round (shard recovery split, short-challenge panic,
# n = 256 distinct messages, edge outcomes), then A/B of GA / J2 lanes (8 vs 16)
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
export GPU_MAX_HW_QUEUES=12
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_shard_batch.py \
  tests/test_rp_short_challenge_gpu.py tests/test_edge_outcomes_gpu.py tests/test_configs_gpu.py > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
bash tools/ab_env.sh r04d 3 "--steps 10 --warmup 2" "" "FSDKR_GA_G=16" "FSDKR_J2_G=16" "FSDKR_GA_G=16 FSDKR_J2_G=16" || exit 1
