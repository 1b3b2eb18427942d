#!/bin/bash
# Event counts (COUNTS=1 builds) of the previous kernel and the frustum cull at c3 (1080p) and c4 (4K).
set -e
R=$PWD; OUT=$R/gpurun_out/r5counts; mkdir -p $OUT
for L in head_counts frustum_counts; do
  for cfg in "--width 1920 --height 1080 --K 0.25" "--width 3840 --height 2160 --K 0.22"; do
    echo "== $L $cfg"
    SF_LIB_PARTIAL=1 SF_LIB=$R/ablib/$L.so timeout -k 10 120 python3 -u scripts/tile_schedule.py --counts --reps 2 $cfg --out $OUT/t.npy
  done
done > $OUT/counts.txt 2>&1
grep -v amdgpu.ids $OUT/counts.txt
