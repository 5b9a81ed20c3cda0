set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05j
mkdir -p $OUT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=12
bash tools/gpu_round.sh r05j shard64 trace4 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_w8 -o tr -- python3 $R/bench.py --n 64 --t 32 --joins 4 --steps 4 --warmup 1 --emulate-shard 8 --gap-ms 20 > $OUT/trace_w8.log 2>&1) || { echo trace_w8 failed; tail -20 $OUT/trace_w8.log; exit 1; }
f=$(find $OUT/trace_w8 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/prof_summary.py "$f" --gap 10 --step -1 > $OUT/trace_w8_summary.txt
