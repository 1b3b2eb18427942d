#!/bin/bash
# The root's children built once per wave (table(0) kept across its tiles): GPU suite, then A/B + PMC.
set -e
R=$PWD; OUT=$R/gpurun_out/r5rootc; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
REPS=5 PMC=1 timeout -k 10 900 scripts/lib_ab.sh r5rootc_ab "" ablib/cur.so ablib/rootc.so > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab.txt | grep -v "sf_order\|SQ_ACTIVE_INST_LDS  *1[0-9][0-9]\.\|SQ_BUSY_CYCLES  *1[0-9][0-9][0-9][0-9]\.\|SQ_INSTS_LDS  *1[0-9][0-9]\.0\|SQ_LDS_IDX\|SQ_BUSY"
