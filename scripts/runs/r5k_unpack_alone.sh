#!/bin/bash
set -e
OUT=gpurun_out/r5k; mkdir -p $OUT
for V in 1 0 1 0; do
  SF_UNPACK_V1=$V timeout -k 10 120 python3 -u scripts/unpack_probe.py 3840 2160 0.22 8 50 >> $OUT/unpack_alone.txt 2>&1
  SF_UNPACK_V1=$V timeout -k 10 120 python3 -u scripts/unpack_probe.py 1920 1080 0.25 8 100 >> $OUT/unpack_alone.txt 2>&1
done
grep -v amdgpu.ids $OUT/unpack_alone.txt
