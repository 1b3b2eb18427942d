#!/bin/bash
# LLVM AMDGPU scheduling strategies for the library (same sources): A/B + PMC against the default build.
set -e
R=$PWD; OUT=$R/gpurun_out/r5sched; mkdir -p $OUT
REPS=4 PMC=1 timeout -k 10 1000 scripts/lib_ab.sh r5sched_ab "" ablib/cur.so ablib/milp.so ablib/iilp.so ablib/mmc.so ablib/trk.so > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab.txt | grep -v "sf_order\|SQ_ACTIVE_INST_LDS  *1[0-9][0-9]\.\|SQ_BUSY_CYCLES  *1[0-9][0-9][0-9][0-9]\.\|SQ_INSTS_LDS  *1[0-9][0-9]\.0"
