#!/bin/bash
# round 6: own-queue context streams after many contexts were made and destroyed (does the process keep their queues?),
# and the torch-free share probe again
set -o pipefail
O=gpurun_out/${TAG:-r6churn}; mkdir -p $O
for pre in "churn40" "churn100" "main,c4,n2,n4"; do
  echo -n "PRE=$pre: " | tee -a $O/churn.txt
  PRE=$pre timeout -k 10 250 python3 -u scripts/member_share_probe.py 8 600 1 2>&1 | grep "N=8 slots" | cut -c1-70 | tee -a $O/churn.txt || exit 1
done
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | tee -a $O/churn.txt || exit 1
done
