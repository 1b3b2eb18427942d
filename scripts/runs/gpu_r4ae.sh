#!/bin/bash
# Round 4: lanes 41..63 repeating child 8 centre (dup8) against final2 (repeating children (lane-32)%9): timing, PMC (bank conflicts).
# (cull_t, reloaded only when maxd grows) against the previous commit (carry.so): parity on the tree (r2c_cull),
# interleaved timing, PMC of each.
R=$PWD; OUT=$R/gpurun_out/r4ae; mkdir -p $OUT
true
true
REPS=3 PMC=1 bash scripts/lib_ab.sh r4ae/ab "" sphereflake-raytracer_amd/build_ab/final2.so sphereflake-raytracer_amd/build_ab/dup8.so
