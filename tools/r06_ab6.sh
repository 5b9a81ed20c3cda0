#!/bin/bash
# round 6: GA padded to whole waves only at 4096 bits (NP) against NF: the collect /
# configs / timed-path / config4 parity suites with NP, configs[4] interleaved, NP's configs[4] timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06o_nopad; mkdir -p $O
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=12
FSDKR_LIB=$R/abtmp/NP.so timeout -k 10 900 python -u -m pytest $R/tests/test_configs_gpu.py $R/tests/test_config4_full_gpu.py \
  $R/tests/test_collect_gpu.py $R/tests/test_timed_path_gpu.py -m gpu -x -v --timeout 400 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_libs.sh r06o_nopad/ab 2 "python bench.py --steps 3 --warmup 1 --no-cpu-baseline --config3-steps 0 --session-steps 3" \
  abtmp/NF.so abtmp/NP.so || exit 1
(cd /tmp && FSDKR_LIB=$R/abtmp/NP.so timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace4 -o tr \
   -- python3 $R/tools/prof_collect.py --full --sessions 1024 --steps 2 > $O/trace4.log 2>&1) || { echo trace4 failed; exit 1; }
f=$(find $O/trace4 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/prof_summary.py "$f" --gap 19 --step -1 > $O/trace4_summary.txt || exit 1
