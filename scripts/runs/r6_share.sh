#!/bin/bash
# round 6: a member's share over N = 1/2/4/8 with every N at the bench's own frames-in-flight policy,
# so the N = 1 basis is the bench's single-GPU period; 1080p and 4K, twice each
set -o pipefail
O=gpurun_out/${TAG:-r6share2}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | tee -a $O/share_1080.txt || exit 1
  timeout -k 10 300 python3 -u scripts/share_probe.py 3840 2160 0.22 2>&1 | grep -v amdgpu.ids | tee -a $O/share_4k.txt || exit 1
done
