#!/bin/bash
# round 6: spread of the 1080p share over 8 -- 12 repetitions of the 20-step and 200-step loops per configuration:
# hardware queues 4 / 8 / 16, one launch per frame at 4 / 8 slots, launches of 8 frames at 16 slots
set -o pipefail
O=gpurun_out/${TAG:-r6sv}; mkdir -p $O
for q in 4 8 16; do
  echo "== GPU_MAX_HW_QUEUES=$q" | tee -a $O/variance.txt
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --reps 12 --configs 4:1,8:1,16:8 2>&1 | grep -v amdgpu.ids | tee -a $O/variance.txt || exit 1
done
