#!/bin/bash
# round-6: configs[4] with the one-wave setup for the prestart's table chains only (D) against
# the group setup everywhere (A); n = 64 with pdl_u1 at issue priority 1 (B) and 3 (C)
set -o pipefail
bash tools/ab_libs.sh r06h_ab_c4_wave_fb 2 "python bench.py --steps 1 --warmup 1 --no-cpu-baseline --config3-steps 0 --session-steps 3" \
  abtmp/A_group.so abtmp/D_wave_fb.so || exit 1
bash tools/ab_libs.sh r06i_ab_u1_prio 3 "python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sessions 0 --config3-steps 0" \
  abtmp/B_wave.so abtmp/C_u1prio3.so || exit 1
