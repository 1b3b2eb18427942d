#!/bin/bash
set -e
mkdir -p gpurun_out/r5knobs; REPS=2 timeout -k 10 1000 scripts/knob_sweep.sh r5knobs "|" "SF_PRIO_BUCKETS=0|" "SF_PRIO_BUCKETS=4|" "SF_PRIO_BUCKETS=12|" "SF_QUEUES_PER_XCD=2|" "SF_QUEUES_PER_XCD=1|" "|--slots 4" "SF_ORDER_EVERY=16|" "SF_ORDER=0|" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5knobs/sweep.txt
