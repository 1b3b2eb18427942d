#!/bin/bash
# round 6: the multi-frame launch over 1/8 shares WITH the heavy-first order (the round-6 share batches ran row-major:
# their "heads" were the first rows, not the heaviest tiles); per-frame launches beside it
set -o pipefail
O=gpurun_out/${TAG:-r6fo}; mkdir -p $O
run() { echo "== $1" | tee -a $O/frames_order.txt; shift; timeout -k 10 300 env "$@" 2>&1 | grep -v amdgpu.ids | tee -a $O/frames_order.txt || exit 1; }
P="python3 -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --reps 3 --configs 4:1,8:8,16:8"
run "row-major (default)" $P
run "ordered, rebuilt every 64th, no recording between" SF_ORDER=1 SF_ORDER_EVERY=64 SF_ORDER_RECORD=0 $P
run "ordered, every 8th" SF_ORDER=1 SF_ORDER_EVERY=8 SF_ORDER_RECORD=0 $P
run "ordered every 64th, heads 256/frame" SF_ORDER=1 SF_ORDER_EVERY=64 SF_ORDER_RECORD=0 SF_FRAMES_HEAVY=256 $P
