#!/bin/bash
# Round 4: where the trace kernel's time goes -- the stamp build's segment shares and the counts build's events,
# 1080p config view (diagnostic builds, never the product library).
R=$PWD; OUT=$R/gpurun_out/r4s; mkdir -p $OUT
SF_LIB=$R/sphereflake-raytracer_amd/build_phases/libsphereflake_hip.so timeout -k 10 120 python3 -u scripts/tile_schedule.py --reps 3 --out $OUT/phases.npy > $OUT/phases.txt 2>&1 || { tail -5 $OUT/phases.txt; exit 5; }
grep -v amdgpu $OUT/phases.txt
SF_LIB=$R/sphereflake-raytracer_amd/build_counts/libsphereflake_hip.so timeout -k 10 120 python3 -u scripts/tile_schedule.py --reps 3 --counts --out $OUT/counts.npy > $OUT/counts.txt 2>&1 || { tail -5 $OUT/counts.txt; exit 6; }
grep -v amdgpu $OUT/counts.txt
