#!/bin/bash
# round 6: the 1080p share over 8 at 4 in flight -- row-major against the heavy-first order with / without raised
# wave priority and with split heavy buckets, stale (rebuilt every 64th, no recording between) or every 4th
set -o pipefail
O=gpurun_out/${TAG:-r6so}; mkdir -p $O
run() { echo "== $1" | tee -a $O/share_order.txt; shift; PROBE_N=8 timeout -k 10 300 env "$@" python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | tee -a $O/share_order.txt || exit 1; }
for r in 1 2; do
run "row-major"
run "order stale, prio on" SF_ORDER=1 SF_ORDER_EVERY=64 SF_ORDER_RECORD=0
run "order stale, prio off" SF_ORDER=1 SF_ORDER_EVERY=64 SF_ORDER_RECORD=0 SF_PRIO_BUCKETS=0
run "order stale, prio off, top 2 buckets split in 4" SF_ORDER=1 SF_ORDER_EVERY=64 SF_ORDER_RECORD=0 SF_PRIO_BUCKETS=0 SF_SPLIT_BUCKETS=2 SF_SPLIT_PARTS=4
run "order stale, prio off, top 4 buckets split in 4" SF_ORDER=1 SF_ORDER_EVERY=64 SF_ORDER_RECORD=0 SF_PRIO_BUCKETS=0 SF_SPLIT_BUCKETS=4 SF_SPLIT_PARTS=4
run "order every 4th, prio off, top 2 split" SF_ORDER=1 SF_ORDER_EVERY=4 SF_ORDER_RECORD=0 SF_PRIO_BUCKETS=0 SF_SPLIT_BUCKETS=2 SF_SPLIT_PARTS=4
done
