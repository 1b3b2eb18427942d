#!/bin/bash
# Diagnostics: traversal event counts + lane utilisation (COUNTS=1 build) and the per-tile schedule of the
# product build, at c3 and c1. Usage (on the box, repo root): scripts/lane_probe.sh <tag>
set -e
OUT=gpurun_out/${1:-lanes}; mkdir -p $OUT
CL=$PWD/sphereflake-raytracer_amd/build_counts/libsphereflake_hip.so
SF_LIB=$CL timeout -k 10 120 python scripts/tile_schedule.py --reps 2 --counts --out $OUT/c3_counts.npy > $OUT/c3_counts.txt 2>&1
SF_LIB=$CL timeout -k 10 120 python scripts/tile_schedule.py --reps 2 --counts --width 640 --height 360 --K 1.0 --out $OUT/c1_counts.npy > $OUT/c1_counts.txt 2>&1
timeout -k 10 120 python scripts/tile_schedule.py --reps 3 --out $OUT/c3_trace.npy > $OUT/c3_trace.txt 2>&1
grep -hv amdgpu.ids $OUT/*.txt
