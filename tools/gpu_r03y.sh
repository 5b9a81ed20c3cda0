#!/bin/bash
# configs[4] host cost on the GPU box: SessionSet pack (fresh vs pre-touched
# buffers, host only) and the multi-session prepare phases.
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03y; mkdir -p $O
timeout -k 10 300 python $R/tools/pack_many_cpu.py --split --reps 3 > $O/pack.jsonl 2>&1 || { echo "pack failed"; tail $O/pack.jsonl; exit 1; }
FSDKR_PREP_PROFILE=1 timeout -k 10 400 python $R/tools/phases_many.py --reps 2 > $O/phases.jsonl 2> $O/prep.txt || { echo "phases failed"; tail -20 $O/prep.txt; exit 1; }
echo "all ok"
