#!/bin/bash
# Round 4: lanes 27..31 repeat axis builders instead of child 0 centre (lane32b) against lane32: parity, timing, PMC.
# (cull_t, reloaded only when maxd grows) against the previous commit (carry.so): parity on the tree (r2c_cull),
# interleaved timing, PMC of each.
R=$PWD; OUT=$R/gpurun_out/r4x; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 5; }
tail -2 $OUT/pytest_gpu.log
REPS=3 PMC=1 bash scripts/lib_ab.sh r4x/ab "" sphereflake-raytracer_amd/build_ab/lane32.so sphereflake-raytracer_amd/build_ab/lane32b.so
