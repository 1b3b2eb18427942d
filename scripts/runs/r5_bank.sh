#!/bin/bash
# Centre-lane remap (child 8 stored from the low lane group): GPU suite on the in-tree library, then A/B + PMC.
set -e
OUT=gpurun_out/r5bank; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
REPS=3 PMC=1 scripts/lib_ab.sh r5bank "" ablib/base.so ablib/bank.so
