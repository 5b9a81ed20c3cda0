#!/bin/bash
# round 6: no in-cycle carry folds for the L = 27 shapes (NF: 3072-bit 4-lane, 6144-bit 8-lane)
# against HEAD (U3): parity suites of those shapes with NF, then configs[4] interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06n_nofold; mkdir -p $O
FSDKR_LIB=$R/abtmp/NF.so timeout -k 10 900 python -u -m pytest $R/tests/test_modexp_gpu.py $R/tests/test_fixedbase_gpu.py \
  $R/tests/test_configs_gpu.py $R/tests/test_config4_full_gpu.py $R/tests/test_golden_gpu.py -m gpu -x -v --timeout 400 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_libs.sh r06n_nofold/ab 2 "python bench.py --steps 3 --warmup 1 --no-cpu-baseline --config3-steps 0 --session-steps 3" \
  abtmp/U3.so abtmp/NF.so || exit 1
