#!/bin/bash
# Child-loop constants carried in SGPRs (LOD threshold, far bound): GPU suite, then A/B + PMC against the previous kernel.
set -e
R=$PWD; OUT=$R/gpurun_out/r5cc; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
REPS=4 PMC=1 timeout -k 10 600 scripts/lib_ab.sh r5cc_ab "" ablib/head.so ablib/cc.so ablib/cc2.so > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab.txt | grep -v "sf_order\|SQ_ACTIVE_INST_LDS *1\|SQ_BUSY_CYCLES *1[0-9][0-9][0-9][0-9]\.\|SQ_INSTS_LDS *1[0-9][0-9]\.0"
