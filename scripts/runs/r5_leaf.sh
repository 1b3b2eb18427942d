#!/bin/bash
# Leaf test at child entry (no per-level leaf mask in the stack), back children at bits 16+: GPU suite + A/B + PMC.
set -e
OUT=gpurun_out/r5leaf; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
REPS=3 PMC=1 scripts/lib_ab.sh r5leaf "" ablib/base.so ablib/leaf.so
