#!/bin/bash
# round 6: GA lanes for 8 193-16 384 chains (the emulated 8-way n = 256 rank's 16 384):
# 16 (HEAD) against 8 (GA8), interleaved whole rank-0 calls; n = 64 (7 680 chains) as
# a control that both builds run identically
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/ab_libs.sh r06z_ga8/s8 3 "python $R/bench.py --n 256 --t 128 --joins 0 --steps 5 --warmup 1 --emulate-shard 8" \
  $R/abtmp/HEAD.so $R/abtmp/GA8.so || exit 1
bash $R/tools/ab_libs.sh r06z_ga8/s4 1 "python $R/bench.py --n 256 --t 128 --joins 0 --steps 3 --warmup 1 --emulate-shard 4" \
  $R/abtmp/HEAD.so $R/abtmp/GA8.so || exit 1
