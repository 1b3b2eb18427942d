#!/bin/bash
set -o pipefail
OUT=$PWD/gpurun_out/${1:-r6i}
mkdir -p $OUT
export TMPDIR=/tmp
SF_FRAMES_ONE=1 SF_FRAMES_HEAVY=0 timeout -k 10 200 python -u scripts/frames_probe.py 1920 1080 0.25 --configs "3:1,3:-1,1:1,1:-1" > $OUT/probe_one.txt 2>&1
rc=$?; grep share $OUT/probe_one.txt; [ $rc -ne 0 ] && exit $rc
SF_FRAMES_ONE=1 SF_FRAMES_HEAVY=0 timeout -k 10 200 python -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --configs "4:1,4:-1,1:1,1:-1" > $OUT/probe_one_share8.txt 2>&1
rc=$?; grep share $OUT/probe_one_share8.txt; exit $rc
