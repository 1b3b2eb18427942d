#!/bin/bash
# Schedule study: per-tile durations of the full 8x8 tiles and of each half unit (pixel rows 0-3 / 4-7)
# via the diagnostic SF_FLAG_DIAG_HALF* flags. Usage (on the GPU box, from the repo root).
set -e
OUT=gpurun_out/half; mkdir -p $OUT
for v in "full:0" "r0:4" "r1:12"; do
  n=${v%%:*}; f=${v##*:}
  SF_SPLIT_BUCKETS=0 SF_FLAGS=$f timeout -k 10 120 python3 scripts/tile_schedule.py --reps 3 --out $OUT/$n.npy | grep -v amdgpu.ids | sed "s/^/$n /"
done
