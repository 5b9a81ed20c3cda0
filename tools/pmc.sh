#!/bin/bash
# PMC passes over the metric-2 modexp launch (65 536 x 4096-bit modexp, exponent N,
# modulus N^2), one rocprofv3 run per counter group (gfx950 slot limits: FETCH_SIZE
# and WRITE_SIZE never share a pass).  Usage (via gpurun): bash tools/pmc.sh TAG [--keyed]
# (--keyed: the exponent-per-key launch, modexp_slide_kernel)
set -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
CMD="python3 $R/tools/bench_modexp.py --count 65536 --reps 1 --widths 128 $2"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter listing failed rc=$?"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- $CMD \
    > $OUT/$name.log 2>&1 || { echo "pass $name failed rc=$?"; tail -20 $OUT/$name.log; exit 1; }
  echo "pass $name ok"
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
pass sq2 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32
pass l2 TCC_HIT_sum TCC_MISS_sum
