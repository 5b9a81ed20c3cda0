set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_inverse_gpu.py tests/test_negative_operands_gpu.py tests/test_edge_outcomes_gpu.py tests/test_collect_gpu.py tests/test_shard_batch.py > gpurun_out/r05x_tests.txt 2>&1 || { tail -30 gpurun_out/r05x_tests.txt; exit 1; }
tail -3 gpurun_out/r05x_tests.txt
bash tools/ab_env.sh r05x_ab_batch_inv 3 "" "FSDKR_BATCH_INV=0" "" || exit 1
