#!/bin/bash
# round 6: is the slow 1/8 share after other dists a matter of the memory they freed? (PRE=mem<k>: a k-context
# dist's G-buffers allocated and freed through torch, no stream; then the share fresh)
set -o pipefail
O=gpurun_out/${TAG:-r6mem}; mkdir -p $O
for pre in ${PRES:-"mem3" "mem4" "" "mem8" "n2"}; do
  echo -n "PRE=$pre: " | tee -a $O/mem.txt
  PRE=$pre timeout -k 10 200 python3 -u scripts/member_share_probe.py 8 600 1 2>&1 | grep "N=8 slots" | cut -c1-110 | tee -a $O/mem.txt || exit 1
done
