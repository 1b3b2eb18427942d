#!/bin/bash
# Unit-level schedules (SF_FLAG_DIAG_UNITS) at c3 under split variants. Usage: scripts/split_sched.sh <tag> "ENV=.." ...
set -e
OUT=gpurun_out/${1:-ss}; shift; mkdir -p $OUT
i=0
for v in "$@"; do
  i=$((i+1))
  env SF_FLAGS=0x20 $v timeout -k 10 120 python3 scripts/tile_schedule.py --reps 3 --out $OUT/c3_v$i.npy 2>&1 | grep -v amdgpu.ids | sed "s/^/c3 $v /"
done
