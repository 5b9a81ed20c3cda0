#!/bin/bash
# round 6: reserved CUs for a small call's latency-bound jobs (Ctx::kLatCus = 16:
# GA on 240 CUs, the few-wave serial jobs on the other 16, throughput jobs anywhere)
# against the same source with kLatCus = 0: the collect / timed-path / shard suites
# on the variant, then interleaved n = 64 lines and one emulated 8-way n = 64 rank
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zc_lat; mkdir -p $O
FSDKR_LIB=$R/abtmp/LAT16.so timeout -k 10 600 python -u -m pytest $R/tests/test_collect_gpu.py $R/tests/test_timed_path_gpu.py \
  $R/tests/test_shard_collect.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_libs.sh r06zc_lat/ab 4 "python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0" \
  abtmp/A.so abtmp/LAT16.so || exit 1
