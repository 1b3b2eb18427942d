#!/bin/bash
# Round 4: the fused SSAO pass at 7 (68 VGPRs) vs 8 waves per SIMD (64 VGPRs), interleaved.
R=$PWD; OUT=$R/gpurun_out/r4q; mkdir -p $OUT
for rep in 1 2 3; do
  for w in 0 1; do
    SF_POST_W8=$w timeout -k 10 120 python3 -u scripts/post_probe.py > $OUT/p_w$w.txt 2>&1 || { tail -5 $OUT/p_w$w.txt; exit 6; }
    echo "w8=$w $(grep 'post fused' $OUT/p_w$w.txt | cut -c1-40)"
  done
done
SF_POST_W8=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_post.py > $OUT/pytest_w8.log 2>&1 || { tail -20 $OUT/pytest_w8.log; exit 5; }
tail -1 $OUT/pytest_w8.log
