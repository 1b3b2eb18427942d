#!/bin/bash
# round 6: the 1080p share over 8 at the bench's policy, in a process with and without torch's runtime initialised
set -o pipefail
O=gpurun_out/${TAG:-r6stq}; mkdir -p $O
for r in 1 2 3; do
  for t in "" 1; do
    echo -n "torch=${t:-0}: " | tee -a $O/share_torch.txt
    PROBE_TORCH=$t PROBE_N=8 timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | sed 's/.*\]: //' | tee -a $O/share_torch.txt || exit 1
  done
done
