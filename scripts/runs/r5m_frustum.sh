#!/bin/bash
# Tile-frustum plane-pair cull of deep expansions: GPU parity suite, then A/B against the previous kernel
# (timing lines interleaved, one PMC pass each).
set -e
R=$PWD; OUT=$R/gpurun_out/r5frustum; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
REPS=3 PMC=1 timeout -k 10 600 scripts/lib_ab.sh r5frustum_ab "" ablib/head.so ablib/frustum.so > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
