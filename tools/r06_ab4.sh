#!/bin/bash
# round 6: pdl_u1 at issue priority 3 (U3) against HEAD (H): n = 64 timeline with U3,
# interleaved n = 64 bench lines, then the metric-2 PMC passes (keyed launch) at HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06k_u1prio; mkdir -p $O
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=12
(cd /tmp && FSDKR_LIB=$R/abtmp/U3.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr \
   -- python3 $R/tools/prof_collect.py --full --steps 4 > $O/trace.log 2>&1) || { echo trace failed; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/prof_summary.py "$f" --gap 10 --step -2 > $O/trace_summary.txt || exit 1
bash tools/ab_libs.sh r06k_u1prio/ab 3 "python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0" \
  abtmp/H.so abtmp/U3.so || exit 1
FSDKR_LIB=$R/abtmp/H.so bash tools/pmc.sh r06k_u1prio/pmcmx --keyed || exit 1
