#!/bin/bash
# Lone-frame unit traces with and without subtree-split tiles (scripts/latency_probe.py, SF_FLAG_DIAG_UNITS).
set -e
OUT=gpurun_out/r5sublat; mkdir -p $OUT
SF_FLAGS=0x20 timeout -k 10 120 python3 -u scripts/latency_probe.py > $OUT/lat_base.txt 2>&1; grep frame $OUT/lat_base.txt
SF_FLAGS=0x20 SF_SPLIT_PARTS=subtree SF_SPLIT_BUCKETS=model timeout -k 10 120 python3 -u scripts/latency_probe.py > $OUT/lat_sub.txt 2>&1; grep frame $OUT/lat_sub.txt
SF_FLAGS=0x20 SF_SPLIT_PARTS=subtree SF_SPLIT_BUCKETS=model SF_SPLIT_DEPTH=5 timeout -k 10 120 python3 -u scripts/latency_probe.py > $OUT/lat_sub5.txt 2>&1; grep frame $OUT/lat_sub5.txt
