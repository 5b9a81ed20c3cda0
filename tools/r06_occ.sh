#!/bin/bash
# GA-shaped 4096-bit modexp alone (exponent N per key, sliding windows, and per-instance
# exponent rows) at 0.9 / 1.9 / 4 / 7.5 waves per SIMD for 16, 8 and 32 lanes per chain
set -o pipefail
O=gpurun_out/r06l_occ; mkdir -p $O
for c in 3840 7680 16384 30720; do
  timeout -k 10 200 python tools/bench_modexp.py --count $c --reps 3 --widths 128 --groups 16,8,32 --keyed >> $O/keyed.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 200 python tools/bench_modexp.py --count $c --reps 3 --widths 128 --groups 16,8 >> $O/rows.jsonl 2>> $O/err.log || exit 1
  echo "count $c done"
done
