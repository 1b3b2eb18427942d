#!/bin/bash
# 8 tile queues per XCD (less ticket contention per queue word) against 4: GPU suite, bench lines, lone frames.
set -e
R=$PWD; OUT=$R/gpurun_out/r5q8; mkdir -p $OUT
true
true
REPS=4 timeout -k 10 900 scripts/knob_sweep.sh r5q8 "SF_QUEUES_PER_XCD=4|" "SF_QUEUES_PER_XCD=8|" > $OUT/sweep.txt 2>&1 || { tail -5 $OUT/sweep.txt; exit 1; }
grep -v amdgpu.ids $OUT/sweep.txt
for rep in 1 2; do for q in 4 8; do
  echo -n "q$q "; SF_QUEUES_PER_XCD=$q timeout -k 10 120 python3 -u scripts/lone_latency.py 300 2>&1 | grep "lone frame"
done; done
