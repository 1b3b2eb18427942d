#!/bin/bash
# Round 4: a 1080p member's share over 8 GPUs (one GPU, 3 frames in flight) under launch-shape knobs.
R=$PWD; OUT=$R/gpurun_out/r4g; mkdir -p $OUT
for rep in 1 2; do
for v in "base SF_NOP=1" "pipe0 SF_PIPE=0" "waves1 SF_TRACE_WAVES=1" "waves4 SF_TRACE_WAVES=4" "nonpers SF_PERSISTENT=0" "prio0 SF_PRIO_BUCKETS=0" "q1 SF_QUEUES_PER_XCD=1"; do
  set -- $v; name=$1; shift
  env "$@" PROBE_STEPS=600 PROBE_N=8 PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 200 python3 -u scripts/share_probe.py > $OUT/share_$name.txt 2>&1 || { tail -3 $OUT/share_$name.txt; exit 6; }
  echo "$name: $(grep slots $OUT/share_$name.txt | tr '\n' ' ')"
done
done
