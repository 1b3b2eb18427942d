#!/bin/bash
# round 6: the 1/8 share after dists of other slot counts were made and closed (their streams' hardware queues are
# then reused): which sequences leave it slow
set -o pipefail
O=gpurun_out/${TAG:-r6reuse}; mkdir -p $O
for pre in "warm" "n8,n4" "n16" "n2" "warm,n8"; do
  echo "PRE=$pre" | tee -a $O/reuse.txt
  PRE=$pre timeout -k 10 200 python3 -u scripts/member_share_probe.py 8 600 1 2>&1 | grep -v amdgpu.ids | grep "N=8 slots" | cut -c1-80 | tee -a $O/reuse.txt || exit 1
done
