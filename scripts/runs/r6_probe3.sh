#!/bin/bash
set -o pipefail
OUT=$PWD/gpurun_out/${1:-r6h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_frames.txt 2>&1
rc=$?; tail -2 $OUT/pytest_frames.txt; [ $rc -ne 0 ] && exit $rc
SF_FRAMES_HEAVY=64 timeout -k 10 200 python -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --configs "4:1,8:8,16:8,8:4" > $OUT/probe_share8.txt 2>&1
rc=$?; grep share $OUT/probe_share8.txt; [ $rc -ne 0 ] && exit $rc
SF_FRAMES_HEAVY=64 timeout -k 10 200 python -u scripts/frames_probe.py 1920 1080 0.25 --configs "3:1,8:4,16:8" > $OUT/probe_1080.txt 2>&1
rc=$?; grep share $OUT/probe_1080.txt; exit $rc
