#!/bin/bash
# Interleaved A/B/C... of environment settings on one box: bench.py's n = 64
# whole collect() step (same build, same inputs), variants alternated per round.
# Usage (via gpurun): bash tools/ab_env.sh TAG ROUNDS "EXTRA BENCH ARGS" "ENV_0" "ENV_1" ...
#   ENV_k: space-separated VAR=value assignments ("" for the baseline)
# Output: gpurun_out/TAG/bench_v<k>.jsonl (one bench line per run)
set -o pipefail
TAG=$1; ROUNDS=$2; EXTRA=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  k=0
  for envs in "$@"; do
    echo "$envs" > $O/v$k.env
    timeout -k 10 200 env $envs python bench.py --no-cpu-baseline --sessions 0 --config3-steps 0 $EXTRA \
      >> $O/bench_v$k.jsonl 2>> $O/bench_v$k.err || { echo "variant $k failed"; tail -5 $O/bench_v$k.err; exit 1; }
    echo "round $r variant $k done"
    k=$((k + 1))
  done
done
