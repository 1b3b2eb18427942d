#!/bin/bash
# Round 4: a 1080p member's share over 8 GPUs (one GPU) against the frames in flight and launch-shape knobs
# (the grid is under-filled by one share's 4080 tiles: more frames in flight may fill it).
R=$PWD; OUT=$R/gpurun_out/r4h; mkdir -p $OUT
for rep in 1 2; do
for v in "base SF_NOP=1" "pipe0 SF_PIPE=0" "pipe1 SF_PIPE=1" "prio0 SF_PRIO_BUCKETS=0" "waves1 SF_TRACE_WAVES=1" "q1 SF_QUEUES_PER_XCD=1"; do
  set -- $v; name=$1; shift
  env "$@" PROBE_STEPS=600 PROBE_N=1,8 PROBE_SLOTS=2,3,4,6 PROBE_SPLITS=auto,0 timeout -k 10 240 python3 -u scripts/share_probe.py > $OUT/share_${name}_$rep.txt 2>&1 || { tail -3 $OUT/share_${name}_$rep.txt; exit 6; }
  echo "== $name"; cat $OUT/share_${name}_$rep.txt | grep slots
done
done
