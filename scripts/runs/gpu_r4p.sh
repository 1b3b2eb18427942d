#!/bin/bash
# Round 4: SSAO taps with the short correctly rounded forms -- post tests (exhaustive float sweep, extreme values),
# then the fused pass's time and a kernel trace.
R=$PWD; OUT=$R/gpurun_out/r4p; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_post.py > $OUT/pytest_post.log 2>&1 || { tail -30 $OUT/pytest_post.log; exit 5; }
tail -3 $OUT/pytest_post.log
timeout -k 10 120 python3 -u scripts/post_probe.py > $OUT/post_probe.txt 2>&1 || { tail -5 $OUT/post_probe.txt; exit 6; }
cat $OUT/post_probe.txt | grep -v amdgpu
