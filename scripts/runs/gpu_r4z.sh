#!/bin/bash
# Round 4: levels check on the carried offset and the index-order mask by OR (flagfree) against lane32: parity, timing, PMC.
# (cull_t, reloaded only when maxd grows) against the previous commit (carry.so): parity on the tree (r2c_cull),
# interleaved timing, PMC of each.
R=$PWD; OUT=$R/gpurun_out/r4z; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 5; }
tail -2 $OUT/pytest_gpu.log
REPS=4 PMC=1 bash scripts/lib_ab.sh r4z/ab "" sphereflake-raytracer_amd/build_ab/lane32.so sphereflake-raytracer_amd/build_ab/flagfree.so
