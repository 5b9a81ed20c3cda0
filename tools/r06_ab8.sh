#!/bin/bash
# round 6: the table chains' moduli setup overlapped with their copy (FB) against HEAD:
# parity suites of the prestarted tables with FB, then interleaved n = 64 and configs[4] lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06u_fbsetup; mkdir -p $O
FSDKR_LIB=$R/abtmp/FB.so timeout -k 10 900 python -u -m pytest $R/tests/test_collect_gpu.py $R/tests/test_timed_path_gpu.py \
  $R/tests/test_configs_gpu.py $R/tests/test_config4_full_gpu.py $R/tests/test_fixedbase_gpu.py -m gpu -x -v --timeout 400 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_libs.sh r06u_fbsetup/ab 3 "python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0 --session-steps 3" \
  abtmp/HEAD.so abtmp/FB.so || exit 1
