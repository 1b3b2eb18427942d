#!/bin/bash
# round 6: with the contexts' own queues, does the process still need GPU_MAX_HW_QUEUES=16? the 1/8 share at 8 in
# flight with the runtime's default 4 queues vs 16, fresh and after a 3-slot dist
set -o pipefail
O=gpurun_out/${TAG:-r6cmq}; mkdir -p $O
for q in 4 16; do
  for pre in "" "n2"; do
    echo -n "queues=$q PRE=$pre: " | tee -a $O/hwq.txt
    GPU_MAX_HW_QUEUES=$q SF_HW_QUEUES=0 SLOTS=8 PRE=$pre timeout -k 10 200 python3 -u scripts/member_share_probe.py 8 600 1 2>&1 | grep "N=8 slots" | cut -c1-70 | tee -a $O/hwq.txt || exit 1
  done
done
