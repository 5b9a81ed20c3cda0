#!/bin/bash
# One GPU-box session (run via gpurun from the repo root):
#   bash tools/gpu_round.sh TAG STEP [STEP ...]
# Outputs go to gpurun_out/TAG/.  Steps (each under its own time limit; the
# script stops at the first failing step):
#   tests            the whole -m gpu suite                      -> tests.log
#   tests:F1,F2      those test files only (tests/F1, tests/F2)  -> tests.log
#   smoke            __graft_entry__ build-free smoke             -> smoke.log
#   bench            bench.py (default: n = 64 headline, metric 2, configs[3] n = 256,
#                    configs[4], key generation, CPU baseline)    -> bench.json
#   benchq           bench.py without the CPU baseline            -> bench.json
#   prof             rocprofv3 --kernel-trace --stats of a short bench.py run -> prof/
#   trace            kernel trace of whole n = 64 collect() calls + timeline of one -> trace_summary.txt
#   trace4           the same for whole configs[4] collect_many() calls (1024 sessions) -> trace4_summary.txt
#   trace256         the same for whole n = 256 collect() calls (configs[3])  -> trace256_summary.txt
#   pmc64 | pmc256 | pmc4   one --pmc pass over whole n = 64 / n = 256 collect() calls or
#                    configs[4] collect_many() calls (tools/pmc_step.py) -> pmc_step_n64.json /
#                    pmc_step_n256.json / pmc_step_c4.json (per-call counter totals; with
#                    tools/mac_share.py's per-kernel MAC shares of this build: pmc_mac_per_call)
#   pmc256s8         the same over rank 0 of an emulated 8-way n = 256 shard -> pmc_step_n256s8.json
#   pmcmx            PMC passes over the metric-2 modexp launch (tools/pmc.sh)
#   shard256         bench.py --emulate-shard 2 / 4 / 8 at n = 256 -> shard_n256.jsonl
#   trace256s8       kernel trace of the emulated rank 0 of an 8-way n = 256 shard -> trace256s8_summary.txt
#   trace64s8        the same for rank 0 of an 8-way n = 64 shard       -> trace64s8_summary.txt
#   rt64s8           that rank with HIP runtime and memory-copy traces too -> rt64s8/
#   shard64          the same at n = 64                            -> shard_n64.jsonl
#   rehearse2        bench.py --gpus 2 under torch.distributed.run, both ranks on GPU 0 (gloo) -> rehearse2.json
#   rehearse4        the same with 4 ranks                          -> rehearse4.json
#   anything else    run as a shell command                       -> extra.log
# Interleaved A/B runs: tools/ab_env.sh (environment variants of one build) and
# tools/ab_lib.sh (two builds of libfsdkr.so).
set -o pipefail
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# collect() runs about twelve concurrent streams; rocprofv3's preload initialises
# HIP before bench.py can set this, so export it here (bench.py/conftest set it otherwise)
export GPU_MAX_HW_QUEUES=12
fail() { echo "$1 failed rc=$2"; tail -30 "$3"; exit 1; }
pmc_step() {   # $1 = label, $2.. = pmc_step.py shape args
  local label=$1; shift
  timeout -k 10 300 python $R/tools/pmc_step.py --gen-only --cache /tmp/$label.pkl "$@" > $OUT/pmc_$label.gen.log 2>&1 \
    || fail "pmc $label workload" $? $OUT/pmc_$label.gen.log
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES SQ_ACTIVE_INST_VALU \
     SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
     -d $OUT/pmc_$label -o run -- python3 $R/tools/pmc_step.py --cache /tmp/$label.pkl --steps 2 "$@" \
     > $OUT/pmc_$label.log 2>&1) || fail "pmc $label" $? $OUT/pmc_$label.log
  local f
  f=$(find $OUT/pmc_$label -name "*counter_collection.csv" | head -1)
  python3 $R/tools/mac_share.py --out $OUT/mac_share.json 2> $OUT/mac_share.err || echo "mac_share failed (no llvm-objdump?)"
  if [ -s $OUT/mac_share.json ]; then
    python3 $R/tools/pmc_summary_step.py "$f" 3 --label $label --mac-share $OUT/mac_share.json > $OUT/pmc_step_$label.json || exit 1
  else
    python3 $R/tools/pmc_summary_step.py "$f" 3 --label $label > $OUT/pmc_step_$label.json || exit 1
  fi
}
for step in "$@"; do
  case $step in
    tests) timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -q --timeout 400 --timeout-method thread \
             > $OUT/tests.log 2>&1 || fail tests $? $OUT/tests.log ;;
    tests:*) files=$(echo ${step#tests:} | tr ',' '\n' | sed "s|^|$R/tests/|" | tr '\n' ' ')
             timeout -k 10 900 python -u -m pytest $files -m gpu -x -v --timeout 400 --timeout-method thread \
               > $OUT/tests.log 2>&1 || fail tests $? $OUT/tests.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
             || fail smoke $? $OUT/smoke.log ;;
    bench) timeout -k 10 600 python $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || fail bench $? $OUT/bench.err ;;
    benchq) timeout -k 10 500 python $R/bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
              || fail bench $? $OUT/bench.err ;;
    prof) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench \
             -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1) \
             || fail prof $? $OUT/prof.log ;;
    trace) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o tr \
              -- python3 $R/tools/prof_collect.py --full --steps 4 > $OUT/trace.log 2>&1) || fail trace $? $OUT/trace.log
           f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
           python $R/tools/prof_summary.py "$f" --gap 10 --step -2 > $OUT/trace_summary.txt || exit 1 ;;
    trace4) (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace4 -o tr \
              -- python3 $R/tools/prof_collect.py --full --sessions 1024 --steps 2 > $OUT/trace4.log 2>&1) \
              || fail trace4 $? $OUT/trace4.log
            f=$(find $OUT/trace4 -name "*kernel_trace.csv" | head -1)
            python $R/tools/prof_summary.py "$f" --gap 19 --step -1 > $OUT/trace4_summary.txt || exit 1 ;;
    trace256) (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace256 -o tr \
                -- python3 $R/tools/prof_collect.py --full --n 256 --t 128 --joins 0 --steps 2 > $OUT/trace256.log 2>&1) \
                || fail trace256 $? $OUT/trace256.log
              f=$(find $OUT/trace256 -name "*kernel_trace.csv" | head -1)
              python $R/tools/prof_summary.py "$f" --gap 10 --step -1 > $OUT/trace256_summary.txt || exit 1 ;;
    trace256s8) (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace256s8 -o tr \
                  -- python3 $R/bench.py --n 256 --t 128 --joins 0 --steps 3 --warmup 1 --emulate-shard 8 --gap-ms 60 \
                  > $OUT/trace256s8.log 2>&1) || fail trace256s8 $? $OUT/trace256s8.log
                f=$(find $OUT/trace256s8 -name "*kernel_trace.csv" | head -1)
                python $R/tools/prof_summary.py "$f" --gap 40 --step -1 > $OUT/trace256s8_summary.txt || exit 1 ;;
    trace64s8) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace64s8 -o tr \
                 -- python3 $R/bench.py --steps 4 --warmup 1 --emulate-shard 8 --gap-ms 30 --sessions 0 --config3-steps 0 \
                 > $OUT/trace64s8.log 2>&1) || fail trace64s8 $? $OUT/trace64s8.log
               f=$(find $OUT/trace64s8 -name "*kernel_trace.csv" | head -1)
               python $R/tools/prof_summary.py "$f" --gap 20 --step -1 > $OUT/trace64s8_summary.txt || exit 1 ;;
    rt64s8) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
              -d $OUT/rt64s8 -o tr -- python3 $R/bench.py --steps 3 --warmup 1 --emulate-shard 8 --gap-ms 30 --sessions 0 \
              --config3-steps 0 > $OUT/rt64s8.log 2>&1) || fail rt64s8 $? $OUT/rt64s8.log ;;
    pmc64) pmc_step n64 --n 64 --joins 4 --t 32 ;;
    pmc256) pmc_step n256 --n 256 --joins 0 --t 128 ;;
    pmc256s8) pmc_step n256s8 --n 256 --joins 0 --t 128 --shard 8 ;;
    pmc4) pmc_step c4 --sessions 1024 --seed 2028 ;;
    pmcmx) bash $R/tools/pmc.sh $TAG/pmcmx || exit 1 ;;
    shard256|shard64)
      n=${step#shard}; t=$((n / 2)); j=$([ $n = 64 ] && echo 4 || echo 0)
      for W in 2 4 8; do
        timeout -k 10 300 python $R/bench.py --n $n --t $t --joins $j --steps 5 --warmup 1 --emulate-shard $W \
          >> $OUT/shard_n$n.jsonl 2>> $OUT/shard_n$n.err || fail "shard $W" $? $OUT/shard_n$n.err
      done ;;
    rehearse2)   # bench.py --gpus 2 as the driver launches it, both ranks on GPU 0 over gloo
      FSDKR_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29517 $R/bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
        --sessions 0 --config3-steps 1 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || fail rehearse2 $? $OUT/rehearse2.err ;;
    rehearse4)   # the same with four ranks (shard_range over 4, max over 4 ranks)
      FSDKR_BENCH_REHEARSE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
        --master-addr 127.0.0.1 --master-port 29519 $R/bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline \
        --sessions 0 --config3-steps 1 > $OUT/rehearse4.json 2> $OUT/rehearse4.err || fail rehearse4 $? $OUT/rehearse4.err ;;
    *) timeout -k 10 600 bash -c "$step" > $OUT/extra.log 2>&1 || fail "$step" $? $OUT/extra.log ;;
  esac
  echo "step $step ok"
done
