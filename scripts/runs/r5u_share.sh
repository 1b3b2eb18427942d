#!/bin/bash
# A 1080p member's share over 8 (4 frames in flight): the row-major default against the heavy-first order kept
# stale (no rebuild kernels) with and without splits of the heaviest tiles.
set -e
OUT=$PWD/gpurun_out/r5share; mkdir -p $OUT
run() { echo -n "[$1] "; env $1 PROBE_SLOTS=4 PROBE_N=1,8 PROBE_SPLITS=$2 timeout -k 10 150 python3 -u scripts/share_probe.py 2>&1 | grep -v amdgpu.ids; }
for rep in 1 2; do
  run "SF_NONE=0" auto
  run "SF_ORDER=1 SF_ORDER_EVERY=3" 0
  run "SF_ORDER=1 SF_ORDER_EVERY=100000" 0
  run "SF_ORDER=1 SF_ORDER_EVERY=100000 SF_SPLIT_PARTS=2" 4
  run "SF_ORDER=1 SF_ORDER_EVERY=100000 SF_SPLIT_PARTS=4" 8
  run "SF_ORDER=1 SF_ORDER_EVERY=100000 SF_SPLIT_PARTS=subtree" model
done 2>&1 | tee $OUT/share.txt
