#!/bin/bash
# round 6: comb_exp software pipeline (the next step's table row and schedule index
# read during the current product) against HEAD: the fixed-base / collect / configs
# suites on the variant, then interleaved n = 64 + configs[4] lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zd_pf; mkdir -p $O
FSDKR_LIB=$R/abtmp/PF.so timeout -k 10 900 python -u -m pytest $R/tests/test_fixedbase_gpu.py $R/tests/test_collect_gpu.py \
  $R/tests/test_configs_gpu.py $R/tests/test_timed_path_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_libs.sh r06zd_pf/ab 3 "python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0" \
  abtmp/A.so abtmp/PF.so || exit 1
