#!/bin/bash
# Round 4: the bench's loop sequence with the live clock of each loop (why the first timed loop ran slow).
R=$PWD; OUT=$R/gpurun_out/r4n; mkdir -p $OUT
for v in "3" "4" "3 E" "4 E" "3"; do
  set -- $v
  if [ -n "$2" ]; then export PROBE_EARLY=1; else unset PROBE_EARLY; fi
  timeout -k 10 100 python3 -u scripts/clock_probe2.py $1 >> $OUT/seq.txt 2>&1 || { tail -3 $OUT/seq.txt; exit 6; }
done
grep F= $OUT/seq.txt
