#!/bin/bash
# Round 4: active-ray compaction (SF_COMPACT=1) against the default kernel on the deep configs (c4 depth 9, c5 depth
# 10) and 1080p, interleaved; plus the post tests after the tracker change.
R=$PWD; OUT=$R/gpurun_out/r4r; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_post.py > $OUT/pytest_post.log 2>&1 || { tail -20 $OUT/pytest_post.log; exit 5; }
tail -1 $OUT/pytest_post.log
show() { python3 -c "import json; j=json.loads(open('$1').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('$2', 'frame', j['frame_ms'], 'clk', j['roofline']['clock_mhz_live'], 'steady', p['steady_frame_ms'], 'check', j['check']['bit_exact'])"; }
for rep in 1 2; do
  for cmp in 0 1; do
    SF_COMPACT=$cmp timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --width 3840 --height 2160 --K 0.22 > $OUT/c4_$cmp_$rep.json 2> $OUT/c4_err || { tail -3 $OUT/c4_err; exit 7; }
    show $OUT/c4_$cmp_$rep.json "c4 compact=$cmp"
    SF_COMPACT=$cmp timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-extras --width 16384 --height 16384 --K 0.2 --steps 10 --warmup 3 > $OUT/c5_$cmp_$rep.json 2> $OUT/c5_err || { tail -3 $OUT/c5_err; exit 7; }
    show $OUT/c5_$cmp_$rep.json "c5 compact=$cmp"
    SF_COMPACT=$cmp timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/c3_$cmp_$rep.json 2> $OUT/c3_err || { tail -3 $OUT/c3_err; exit 7; }
    show $OUT/c3_$cmp_$rep.json "c3 compact=$cmp"
  done
done
