#!/bin/bash
# r04c: whole-call kernel trace of the n = 64 collect() at HEAD, and one PMC pass
# over whole calls (tools/pmc_step.py) for the counter-based issue fraction
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c; mkdir -p $O
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
bash $R/tools/gpu_round.sh r04c trace || exit 1
timeout -k 10 200 python $R/tools/pmc_step.py --gen-only --cache /tmp/n64.pkl > $O/gen.log 2>&1 || { tail $O/gen.log; exit 1; }
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/pmc64 -o run -- python3 $R/tools/pmc_step.py --cache /tmp/n64.pkl --steps 2 > $O/pmc64.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc64.log; exit 1; }
f=$(find $O/pmc64 -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_summary_step.py "$f" 3 --label n64 > $O/pmc64_summary.json || exit 1
echo done
