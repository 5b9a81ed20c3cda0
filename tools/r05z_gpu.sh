set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_collect_gpu.py tests/test_timed_path_gpu.py tests/test_fixedbase_gpu.py tests/test_edge_outcomes_gpu.py > gpurun_out/r05z_tests.txt 2>&1 || { tail -30 gpurun_out/r05z_tests.txt; exit 1; }
tail -2 gpurun_out/r05z_tests.txt
bash tools/ab_env.sh r05z_ab_table_split 3 "" "FSDKR_TABLE_SPLIT=0" "" || exit 1
