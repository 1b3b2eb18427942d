#!/bin/bash
# Contention study: per-tile durations of the persistent kernel under env variants (grid caps via
# SF_MAX_BLOCKS, issue priority via SF_PRIO_TILES). Usage (on the GPU box): scripts/contention_study.sh "ENV=.." ...
set -e
OUT=gpurun_out/cont; mkdir -p $OUT
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 120 python3 scripts/tile_schedule.py --reps 2 --out $OUT/v$i.npy | grep -v amdgpu.ids | sed "s/^/$v /"
done
