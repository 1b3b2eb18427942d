#!/bin/bash
# round 6: the 1080p share over 8 at more frames in flight with as many hardware queues (GPU_MAX_HW_QUEUES, <= 32),
# per-frame launches, row-major
set -o pipefail
O=gpurun_out/${TAG:-r6sq}; mkdir -p $O
for r in 1 2; do
  for q in 4 8 16; do
    echo -n "hwq $q: " | tee -a $O/share_queues.txt
    GPU_MAX_HW_QUEUES=$q PROBE_N=8 PROBE_SLOTS=4,6,8,12,16 timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | sed 's/.*\]: //' | tr '\n' ' ' | tee -a $O/share_queues.txt || exit 1
    echo | tee -a $O/share_queues.txt
  done
done
