set -o pipefail
O=gpurun_out/r01y; mkdir -p $O
timeout -k 10 120 python tools/bench_modexp.py --count 1024 --reps 3 --widths 128 --groups 16,32 > $O/mx1024.jsonl 2>&1 || { tail -20 $O/mx1024.jsonl; exit 1; }
grep -o '"count": [0-9]*\|"kernel_ms": [0-9.]*\|"group": [0-9]*' $O/mx1024.jsonl | paste - - -
timeout -k 10 120 python tools/bench_modexp.py --count 7680 --reps 2 --widths 128 --groups 32 > $O/mx7680.jsonl 2>&1 || { tail -20 $O/mx7680.jsonl; exit 1; }
grep -o '"count": [0-9]*\|"kernel_ms": [0-9.]*\|"group": [0-9]*' $O/mx7680.jsonl | paste - - -
timeout -k 10 400 python -u -m pytest tests/test_collect_gpu.py tests/test_shard_batch.py tests/test_golden_gpu.py tests/test_modexp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for w in 8 4 2; do timeout -k 10 200 python tools/ab_collect.py --shard $w --rounds 4 - FSDKR_COLLECT_GA_G=16 > $O/ab$w.log 2>&1 || exit 1; grep -o '"config": "[^"]*"\|"median_ms": [0-9.]*' $O/ab$w.log | paste - - | sed "s/^/w=$w /"; done
