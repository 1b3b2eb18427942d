#!/bin/bash
# round 6: where the contexts' buffers land (SF_PRINT_ADDRS) for a fresh 8-slot share vs after the N = 2 / 4 dists
set -o pipefail
O=gpurun_out/${TAG:-r6addr}; mkdir -p $O
SF_PRINT_ADDRS=1 timeout -k 10 200 python3 -u scripts/member_share_probe.py 8 600 1 > $O/fresh.txt 2>&1 || exit 1
SF_PRINT_ADDRS=1 PRE=n2,n4 timeout -k 10 200 python3 -u scripts/member_share_probe.py 8 600 1 > $O/pre.txt 2>&1 || exit 1
grep -h "N=8" $O/fresh.txt $O/pre.txt
