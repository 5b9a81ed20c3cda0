#!/bin/bash
# round 6: GA's moduli setup overlapped with the pair-row copy in the prestart (MS)
# against HEAD: collect / timed-path / configs / golden / shard parity with MS, then
# interleaved n = 64 bench lines and one configs[4] line each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06t_modsetup; mkdir -p $O
FSDKR_LIB=$R/abtmp/MS.so timeout -k 10 900 python -u -m pytest $R/tests/test_collect_gpu.py $R/tests/test_timed_path_gpu.py \
  $R/tests/test_configs_gpu.py $R/tests/test_golden_gpu.py $R/tests/test_shard_batch.py -m gpu -x -v --timeout 400 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_libs.sh r06t_modsetup/ab 4 "python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0" \
  abtmp/HEAD.so abtmp/MS.so || exit 1
