#!/bin/bash
# round 6: multi-frame launches with 16 hardware queues (two batches in flight on queues of their own)
set -o pipefail
O=gpurun_out/${TAG:-r6f16}; mkdir -p $O
export GPU_MAX_HW_QUEUES=16
timeout -k 10 300 python3 -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --reps 3 --configs 8:1,16:8,16:4 2>&1 | grep -v amdgpu.ids | tee -a $O/frames_16q.txt || exit 1
timeout -k 10 300 python3 -u scripts/frames_probe.py 1920 1080 0.25 --reps 3 --configs 3:1,8:4,16:4 2>&1 | grep -v amdgpu.ids | tee -a $O/frames_16q.txt || exit 1
