#!/bin/bash
# round-6 A/B session: next-digit carry (A base vs B) on the n = 64 step and metric-2 /
# latency modexp shapes, then GA lanes of the emulated 8-way n = 256 rank (B 16 lanes,
# C 8 lanes, D 4 lanes at 16 384 chains)
set -o pipefail
bash tools/ab_lib.sh r06c_ab_nxt abtmp/A.so abtmp/B.so 2 || exit 1
bash tools/ab_libs.sh r06d_ab_w8_lanes 2 "python bench.py --n 256 --t 128 --joins 0 --steps 4 --warmup 1 --emulate-shard 8" \
  abtmp/B.so abtmp/C_l8.so abtmp/D_l4.so || exit 1
