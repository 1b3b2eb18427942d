#!/bin/bash
# round 6: frames in flight for band shares once each slot stream has a queue of its own (N = 4: 4 / 6 / 8; N = 8:
# 8 / 12 / 16; N = 2: 3 / 4)
set -o pipefail
O=gpurun_out/${TAG:-r6oqs}; mkdir -p $O
for cfg in "4 4" "4 6" "4 8" "8 8" "8 12" "8 16" "2 3" "2 4"; do
  set -- $cfg
  echo -n "N=$1 slots=$2: " | tee -a $O/slots.txt
  SLOTS=$2 timeout -k 10 200 python3 -u scripts/member_share_probe.py $1 600 1 2>&1 | grep "slots=" | cut -c1-70 | tee -a $O/slots.txt || exit 1
done
