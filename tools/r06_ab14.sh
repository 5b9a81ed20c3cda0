#!/bin/bash
# round 6: correct-key chains of small batches one instance per wave (ck_lanes,
# modexp_wave_kernel<72,2,64>) against HEAD: the modexp / collect / timed-path /
# shard suites on the variant, then interleaved emulated 8- and 4-way n = 64 ranks
# and the one-GPU n = 64 call (704 chains: unchanged shape)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zj_ck; mkdir -p $O
FSDKR_LIB=$R/abtmp/WV.so timeout -k 10 900 python -u -m pytest $R/tests/test_modexp_gpu.py $R/tests/test_collect_gpu.py \
  $R/tests/test_timed_path_gpu.py $R/tests/test_shard_batch.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_libs.sh r06zj_ck/s8 3 "python bench.py --steps 10 --warmup 2 --emulate-shard 8 --sessions 0 --config3-steps 0" \
  abtmp/A.so abtmp/WV.so || exit 1
bash tools/ab_libs.sh r06zj_ck/s4 2 "python bench.py --steps 10 --warmup 2 --emulate-shard 4 --sessions 0 --config3-steps 0" \
  abtmp/A.so abtmp/WV.so || exit 1
