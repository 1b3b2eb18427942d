#!/bin/bash
# Tile schedules (per-tile durations, span) under subtree-donation variants, c3 and c1.
# Usage (on the box, repo root): scripts/pair_sched.sh <tag> "ENV=.." ...
set -e
OUT=gpurun_out/${1:-ps}; shift; mkdir -p $OUT
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 120 python3 scripts/tile_schedule.py --reps 2 --out $OUT/c3_v$i.npy 2>&1 | grep -v amdgpu.ids | sed "s/^/c3 $v /"
  env $v timeout -k 10 120 python3 scripts/tile_schedule.py --reps 2 --width 640 --height 360 --K 1.0 --out $OUT/c1_v$i.npy 2>&1 | grep -v amdgpu.ids | sed "s/^/c1 $v /"
done
