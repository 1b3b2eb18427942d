#!/bin/bash
# A/B of the in-tree library (ablib/exp.so) against ablib/leaf.so (the round-end library): GPU suite first.
set -e
OUT=gpurun_out/r5exp; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
REPS=3 PMC=1 scripts/lib_ab.sh r5exp "" ablib/leaf.so ablib/exp.so
