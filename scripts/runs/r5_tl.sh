#!/bin/bash
# Lone-frame timeline (scripts/lone_frame_timeline.py): plain run, then under a runtime + kernel + copy trace.
set -e
R=$PWD; OUT=$R/gpurun_out/r5tl; mkdir -p $OUT
timeout -k 10 120 python3 -u scripts/lone_frame_timeline.py > $OUT/plain.txt 2>&1; cat $OUT/plain.txt | grep lone
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/tr -o run -- python3 $R/scripts/lone_frame_timeline.py > $OUT/traced.txt 2>&1
grep lone $OUT/traced.txt
cd $R && python3 scripts/lone_frame_timeline.py --report $OUT/tr > $OUT/report.txt 2>&1; cat $OUT/report.txt
rm -rf $OUT/tr
