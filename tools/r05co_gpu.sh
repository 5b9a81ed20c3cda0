set -o pipefail
timeout -k 10 300 env FSDKR_GA_COOP=1 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_coop_gpu.py tests/test_shard_batch.py > gpurun_out/r05co_tests.txt 2>&1 || { tail -30 gpurun_out/r05co_tests.txt; exit 1; }
tail -2 gpurun_out/r05co_tests.txt
bash tools/ab_env.sh r05co_ab_w8 2 "--n 64 --t 32 --joins 4 --steps 5 --warmup 1 --emulate-shard 8" "FSDKR_GA_COOP=0" "FSDKR_GA_COOP=1" || exit 1
