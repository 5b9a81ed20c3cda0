set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_modexp_gpu.py -k "joint or every_group" > gpurun_out/r05m_tests.txt 2>&1 || { tail -30 gpurun_out/r05m_tests.txt; exit 1; }
tail -2 gpurun_out/r05m_tests.txt
bash tools/ab_env.sh r05m_ab_w8 2 "--n 64 --t 32 --joins 4 --steps 5 --warmup 1 --emulate-shard 8" "" "FSDKR_GA_LANES=16" "FSDKR_GA_LANES=32" || exit 1
bash tools/ab_env.sh r05m_ab_w4 1 "--n 64 --t 32 --joins 4 --steps 5 --warmup 1 --emulate-shard 4" "FSDKR_GA_LANES=16" "FSDKR_GA_LANES=32" || exit 1
