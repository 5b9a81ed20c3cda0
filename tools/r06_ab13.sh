#!/bin/bash
# round 6: more interleaved rounds of the comb_exp software pipeline (r06_ab12.sh):
# n = 64 alone, configs[4] alone, and an n = 64 kernel trace of the variant
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06ze_pf; mkdir -p $O
bash tools/ab_libs.sh r06ze_pf/n64 5 "python bench.py --steps 12 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0" \
  abtmp/A.so abtmp/PF.so || exit 1
bash tools/ab_libs.sh r06ze_pf/c4 3 "python bench.py --steps 2 --warmup 1 --no-cpu-baseline --config3-steps 0 --session-steps 3 --modexp-count 4096" \
  abtmp/A.so abtmp/PF.so || exit 1
(cd /tmp && FSDKR_LIB=$R/abtmp/PF.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr \
   -- python3 $R/tools/prof_collect.py --full --steps 4 > $O/trace.log 2>&1) || { echo trace failed; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python $R/tools/prof_summary.py "$f" --gap 10 --step -2 > $O/trace_summary.txt || exit 1
