#!/bin/bash
# Round-3 HEAD record: metric-2 PMC passes (HBM bytes, SQ split), PMC of the
# n = 64 pipeline kernels, the bench line (reads the fresh PMC file), a
# kernel-trace --stats profile of the bench command, and smoke().
set -o pipefail
export GPU_MAX_HW_QUEUES=12 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03o}
O=$R/gpurun_out/$TAG; mkdir -p $O
bash $R/tools/pmc.sh ${TAG}_pmc || exit 1
python $R/tools/pmc_summary.py $R/gpurun_out/${TAG}_pmc > $O/pmc_modexp4096.json || exit 1
cp $O/pmc_modexp4096.json $R/profiles/${TAG}_pmc_modexp4096.json
rm -rf $R/gpurun_out/${TAG}_pmc/*/ 
(cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU_INT64 --kernel-trace --output-format csv -d $O/pipe -o run -- python3 $R/tools/prof_collect.py --steps 2 > $O/pipe.log 2>&1) || { echo "pipe pmc failed"; tail -20 $O/pipe.log; exit 1; }
python $R/tools/pmc_kernels.py $(find $O/pipe -name "run_counter_collection.csv" | head -1) > $O/pmc_pipeline_kernels.json || exit 1
rm -rf $O/pipe
timeout -k 10 500 python $R/bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log > $O/bench.json
(cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1) || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/bench_kernel_stats.csv
grep '^{"metric"' $O/prof.log > $O/bench_under_rocprof.json
rm -rf $O/prof
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
echo "all ok"
