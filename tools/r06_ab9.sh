#!/bin/bash
# round 6: host-side GA launch path (GBE: group_by_exponent without a comparison sort of
# every instance, N^2 rows on every host thread) against HEAD: the regrouped-job suites
# with GBE, then interleaved n = 64 + configs[3] lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06v_gbe; mkdir -p $O
FSDKR_LIB=$R/abtmp/GBE.so timeout -k 10 900 python -u -m pytest $R/tests/test_collect_gpu.py $R/tests/test_timed_path_gpu.py \
  $R/tests/test_modexp_gpu.py $R/tests/test_golden_gpu.py $R/tests/test_distribute_gpu.py $R/tests/test_configs_gpu.py \
  -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_libs.sh r06v_gbe/ab 3 "python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 2" \
  abtmp/HEAD.so abtmp/GBE.so || exit 1
