#!/bin/bash
# round 6: share batches (multi-frame launch) with the heavy-first order and NO splits (the earlier ordered runs had
# the small-frame default SF_SPLIT_BUCKETS=auto: heavy tiles split into quarters for the idle wave slots)
set -o pipefail
O=gpurun_out/${TAG:-r6fo2}; mkdir -p $O
run() { echo "== $1" | tee -a $O/frames_order2.txt; shift; timeout -k 10 300 env "$@" 2>&1 | grep -v amdgpu.ids | tee -a $O/frames_order2.txt || exit 1; }
P="python3 -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --reps 3 --configs 4:1,8:8,16:8"
run "row-major (default)" $P
run "ordered, no splits, rebuilt every 64th, no recording between" SF_ORDER=1 SF_SPLIT_BUCKETS=0 SF_ORDER_EVERY=64 SF_ORDER_RECORD=0 $P
run "ordered, no splits, no priority" SF_ORDER=1 SF_SPLIT_BUCKETS=0 SF_ORDER_EVERY=64 SF_ORDER_RECORD=0 SF_PRIO_BUCKETS=0 $P
run "ordered, no splits, rebuilt every 8th" SF_ORDER=1 SF_SPLIT_BUCKETS=0 SF_ORDER_EVERY=8 SF_ORDER_RECORD=0 $P
