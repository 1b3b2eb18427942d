#!/bin/bash
# Round 4: the live clock over ~2.5 s of the moving 1080p loop at 3 and 4 frames in flight (DVFS give-back).
R=$PWD; OUT=$R/gpurun_out/r4k; mkdir -p $OUT
for f in 3 4 3; do
  timeout -k 10 120 python3 -u scripts/ramp_probe.py $f 300 > $OUT/ramp_f$f.txt 2>&1 || { tail -3 $OUT/ramp_f$f.txt; exit 6; }
  echo "== F=$f"; grep window $OUT/ramp_f$f.txt | awk 'NR%20==1'
done
