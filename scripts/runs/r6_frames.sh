#!/bin/bash
# Round-6 multi-frame trace and pipelined unpack: GPU tests, the loop-shape probe (1080p, a 1/8 share), the unpack
# A/B against the round-5 library (ablib/r5.so).
set -o pipefail
OUT=gpurun_out/${1:-r6f}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_dist.py tests/test_gpu_group.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_frames.txt 2>&1
rc=$?; tail -5 $OUT/pytest_frames.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u scripts/frames_probe.py 1920 1080 0.25 --configs "3:1,4:4,8:4,6:2,8:8" > $OUT/probe_1080.txt 2>&1
rc=$?; cat $OUT/probe_1080.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --configs "4:1,8:8,16:8" > $OUT/probe_share8.txt 2>&1
rc=$?; cat $OUT/probe_share8.txt; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for L in r5 cur; do
  LIB=$PWD/ablib/$L.so; [ $L = cur ] && LIB=$PWD/sphereflake-raytracer_amd/build/libsphereflake_hip.so
  echo -n "$L "; SF_LIB_PARTIAL=1 SF_LIB=$LIB timeout -k 10 120 python3 -u scripts/unpack_probe.py 3840 2160 0.22 8 50 2>&1 | grep unpack
  echo -n "$L "; SF_LIB_PARTIAL=1 SF_LIB=$LIB timeout -k 10 120 python3 -u scripts/unpack_probe.py 1920 1080 0.25 8 50 2>&1 | grep unpack
done; done | tee $OUT/unpack_ab.txt
