#!/bin/bash
# round 6: small batches (2P <= 4096 GA chains) back on the one-copy prestart order
# (SM) against HEAD: collect / timed-path / shard suites on the variant, then the
# emulated 8-, 4- and 2-way n = 64 ranks, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zm_sm; mkdir -p $O
FSDKR_LIB=$R/abtmp/SM.so timeout -k 10 900 python -u -m pytest $R/tests/test_collect_gpu.py $R/tests/test_timed_path_gpu.py \
  $R/tests/test_shard_batch.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for W in 8 4 2; do
  bash tools/ab_libs.sh r06zm_sm/s$W 3 "python bench.py --steps 10 --warmup 2 --emulate-shard $W --sessions 0 --config3-steps 0" \
    abtmp/A.so abtmp/SM.so || exit 1
done
