#!/bin/bash
# VALU instruction-mix PMC passes over a short bench run (kernel-trace only). Usage: scripts/prof_mix.sh <tag>
set -e
TAG=${1:-mix}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras"
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- $BENCH > $OUT/$name.log 2>&1
}
run m1 SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64
run m2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_WAVE_CYCLES
run m3 SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_SMEM SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_ANY SQ_CYCLES
run g GRBM_GUI_ACTIVE GRBM_COUNT
python3 $R/scripts/pmc_summary.py $OUT/m1 $OUT/m2 $OUT/m3 $OUT/g > $OUT/summary.txt
grep -A30 "== sf_trace_queue2" $OUT/summary.txt | head -32
