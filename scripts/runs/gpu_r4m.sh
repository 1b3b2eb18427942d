#!/bin/bash
# Round 4: the live clock under the bench's settle shape (chunks of 20 + synchronize) vs long chunks, +- torch.
R=$PWD; OUT=$R/gpurun_out/r4m; mkdir -p $OUT
for v in "c20 3 20" "c20t 3 20 T" "c200 3 200" "c20s4 4 20"; do
  set -- $v; name=$1
  if [ -n "$4" ]; then export PROBE_TORCH=1; else unset PROBE_TORCH; fi
  timeout -k 10 100 python3 -u scripts/clock_probe.py $2 $3 1500 > $OUT/$name.txt 2>&1 || { tail -3 $OUT/$name.txt; exit 6; }
  echo "== $name"; grep chunk $OUT/$name.txt | awk 'NR%3==1'
done
