#!/bin/bash
# A 1080p member's share over 8 (4 frames in flight): the persistent grid capped (fewer workgroups per launch)
# and two waves per workgroup, against the default (one wave per tile).
set -e
OUT=$PWD/gpurun_out/r5share2; mkdir -p $OUT
run() { echo -n "[$1] "; env $1 PROBE_SLOTS=4 PROBE_N=1,8 PROBE_SPLITS=auto timeout -k 10 150 python3 -u scripts/share_probe.py 2>&1 | grep -v amdgpu.ids; }
for rep in 1 2; do
  run "SF_NONE=0"
  run "SF_MAX_BLOCKS=4096"
  run "SF_MAX_BLOCKS=2048"
  run "SF_MAX_BLOCKS=1024"
  run "SF_TRACE_WAVES=2"
done 2>&1 | tee $OUT/share.txt
