#!/bin/bash
# The node table built per depth-3 subtree: slab / unpack / dist parity, then the rebuild per view against the previous library.
set -e
R=$PWD; OUT=$R/gpurun_out/r5ntab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "slab or unpack or group or dist" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do for L in cur ntab; do
  echo -n "$L 1080p "; SF_LIB_PARTIAL=1 SF_LIB=$R/ablib/$L.so timeout -k 10 120 python3 -u scripts/node_table_probe.py 1920 1080 0.25 8 40 2>&1 | grep table
  echo -n "$L 4K "; SF_LIB_PARTIAL=1 SF_LIB=$R/ablib/$L.so timeout -k 10 120 python3 -u scripts/node_table_probe.py 3840 2160 0.22 8 40 2>&1 | grep table
done; done | tee $OUT/ntab.txt
