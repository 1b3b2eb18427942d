#!/bin/bash
# Round 4: the traversal with the level's table pointer and depth-constant offset carried across push / pop
# (carry.so = the tree) against the previous build (base.so): parity suite on the tree first, then interleaved
# timing and a PMC pass of each.
R=$PWD; OUT=$R/gpurun_out/r4t; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 5; }
tail -2 $OUT/pytest_gpu.log
REPS=4 PMC=1 bash scripts/lib_ab.sh r4t/ab "" sphereflake-raytracer_amd/build_ab/base.so sphereflake-raytracer_amd/build_ab/carry.so
