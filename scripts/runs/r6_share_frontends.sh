#!/bin/bash
# round 6: the 1/8 share through plain contexts vs sf_dist (lazy view) vs sf_dist with the slot's view set directly,
# 8 in flight on 16 hardware queues, long loops (scripts/share_loop_probe.py)
set -o pipefail
O=gpurun_out/${TAG:-r6sfe}; mkdir -p $O
for r in 1 2; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python3 -u scripts/share_loop_probe.py 8 8 6000 2>&1 | grep -v amdgpu.ids | tee -a $O/frontends.txt || exit 1
done
