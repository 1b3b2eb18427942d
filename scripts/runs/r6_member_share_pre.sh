#!/bin/bash
# round 6: the bench's member-share leg after the legs bench.py runs before it (scripts/member_share_probe.py PRE=...)
set -o pipefail
O=gpurun_out/${TAG:-r6msq}; mkdir -p $O
for pre in "main,c4,n2,n4" "main" "c4" "n2,n4"; do
  echo "PRE=$pre" | tee -a $O/member_share_pre.txt
  PRE=$pre timeout -k 10 300 python3 -u scripts/member_share_probe.py 8 600 2 2>&1 | grep -v amdgpu.ids | tee -a $O/member_share_pre.txt || exit 1
done
