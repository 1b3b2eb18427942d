#!/bin/bash
# Lone-frame latency: the previous library, idle-slot sync skipped, and the polling wait; then the GPU suite.
set -e
R=$PWD; OUT=$R/gpurun_out/r5lat; mkdir -p $OUT
for rep in 1 2 3; do
  for v in head sync sync@1; do
    L=${v%@*}; S=0; [ "$L" != "$v" ] && S=1
    echo -n "$v  "; SF_SYNC_SPIN=$S SF_LIB_PARTIAL=1 SF_LIB=$R/ablib/$L.so timeout -k 10 120 python3 -u scripts/lone_latency.py 300 2>&1 | grep "lone frame"
  done
done > $OUT/lat.txt 2>&1
cat $OUT/lat.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
