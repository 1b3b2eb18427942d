#!/bin/bash
# round 6: the 1080p share over 8 with 16 queues -- the persistent grid capped (each wave more than one tile, the
# per-wave setup amortised) at more frames in flight
set -o pipefail
O=gpurun_out/${TAG:-r6sg}; mkdir -p $O
for r in 1 2; do
  for b in 0 4096 2048; do
    echo -n "max_blocks $b: " | tee -a $O/share_grid.txt
    SF_MAX_BLOCKS=$b PROBE_N=8 PROBE_SLOTS=8,12,16 timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | sed 's/.*\]: //' | tr '\n' ' ' | tee -a $O/share_grid.txt || exit 1
    echo | tee -a $O/share_grid.txt
  done
done
