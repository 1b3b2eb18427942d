#!/bin/bash
# round 6: a 1/8 (and 1/4) band share's persistent grid capped below one workgroup per tile (SF_MAX_BLOCKS), at the
# bench's policy (16 hardware queues, 8 / 4 frames in flight): fewer, longer-lived waves per share frame
set -o pipefail
O=gpurun_out/${TAG:-r6sgc}; mkdir -p $O
for r in 1 2; do
  for mb in 0 1024 2048 3072; do
    if [ $mb = 0 ]; then unset SF_MAX_BLOCKS; else export SF_MAX_BLOCKS=$mb; fi
    PROBE_N=1,4,8 timeout -k 10 200 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | sed "s/^/max_blocks=$mb /" | tee -a $O/grid_cap.txt || exit 1
  done
done
