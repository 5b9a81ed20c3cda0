#!/bin/bash
# r04e: n = 256 (configs[3], distinct messages) GA-lanes A/B (8 / 16 / 4), then the
# emulated 2 / 4 / 8-way shard ranks of n = 256 (rank 0's whole shard.collect call)
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
export GPU_MAX_HW_QUEUES=12
bash tools/ab_env.sh r04e 2 "--n 256 --t 128 --joins 0 --steps 3 --warmup 1" "" "FSDKR_GA_G=16" "FSDKR_GA_G=4" || exit 1
for W in 2 4 8; do
  timeout -k 10 300 python bench.py --n 256 --t 128 --joins 0 --steps 3 --warmup 1 --emulate-shard $W >> $O/shard_n256.jsonl 2>> $O/shard.err || { echo "shard $W failed"; tail -5 $O/shard.err; exit 1; }
  echo "shard $W done"
done
