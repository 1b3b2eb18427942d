#!/bin/bash
# round 6: the bench's member-share leg alone with its host enqueue trace (scripts/member_share_probe.py)
set -o pipefail
O=gpurun_out/${TAG:-r6msp}; mkdir -p $O
timeout -k 10 200 python3 -u scripts/member_share_probe.py 8 600 2 2>&1 | grep -v amdgpu.ids | tee -a $O/member_share.txt || exit 1
timeout -k 10 200 python3 -u scripts/member_share_probe.py 8 3000 1 2>&1 | grep -v amdgpu.ids | tee -a $O/member_share.txt || exit 1
timeout -k 10 200 python3 -u scripts/member_share_probe.py 4 600 1 2>&1 | grep -v amdgpu.ids | tee -a $O/member_share.txt || exit 1
