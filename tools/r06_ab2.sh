#!/bin/bash
# round-6: one-wave-per-modulus 3072-bit setup -- its parity suites, then configs[4]
# whole steps interleaved (A: 4-lane group setup, B: wave setup) and a configs[4] trace
set -o pipefail
bash tools/gpu_round.sh r06f tests:test_modexp_gpu.py,test_fixedbase_gpu.py,test_configs_gpu.py,test_keygen_gpu.py || exit 1
bash tools/ab_libs.sh r06g_ab_c4_wave_setup 2 "python bench.py --steps 1 --warmup 1 --no-cpu-baseline --config3-steps 0 --session-steps 3" \
  abtmp/A_group.so abtmp/B_wave.so || exit 1
bash tools/gpu_round.sh r06f trace4 || exit 1
