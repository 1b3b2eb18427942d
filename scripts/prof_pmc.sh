#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel-trace only: no sys/runtime trace with --pmc)
# over a short bench run. Usage (on the GPU box, from the repo root): scripts/prof_pmc.sh <tag> [bench args]
set -e
TAG=${1:-pmc}; shift || true
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras $*"
run() {  # run <name> <counters...>
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- $BENCH > $OUT/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
run sq3 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
