#!/bin/bash
# Unpack variants: parity of the slab tests, then the unpack alone at 4K and 1080p over 8.
set -e
R=$PWD; OUT=$R/gpurun_out/r5unpack2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "slab or unpack or group or dist" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
timeout -k 10 120 python3 -u scripts/unpack_probe.py 3840 2160 0.22 8 50 | grep unpack
timeout -k 10 120 python3 -u scripts/unpack_probe.py 1920 1080 0.25 8 50 | grep unpack
done > $OUT/unpack_alone.txt 2>&1; grep unpack $OUT/unpack_alone.txt
