#!/bin/bash
# Round 4: one wave per workgroup (SF_TRACE_WAVES=1, sf_trace_queue1) against two (default) with the round-end
# kernel: 1080p x4, 640x360 and 4K x2, interleaved.
R=$PWD; OUT=$R/gpurun_out/r4ah; mkdir -p $OUT
show() { python3 -c "import json; j=json.loads(open('$1').read().strip().split(chr(10))[-1]); print('$2', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'lat', j['frame_latency_ms'], 'clk', j['roofline']['clock_mhz_live'], 'check', j['check']['bit_exact'])"; }
for rep in 1 2 3 4; do
  for w in 2 1; do
    SF_TRACE_WAVES=$w timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 7; }
    show $OUT/b.json "c3 waves$w"
  done
done
for rep in 1 2; do
  for w in 2 1; do
    SF_TRACE_WAVES=$w timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --width 640 --height 360 --K 1.0 > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 7; }
    show $OUT/b.json "c1 waves$w"
    SF_TRACE_WAVES=$w timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --width 3840 --height 2160 --K 0.22 > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 7; }
    show $OUT/b.json "c4 waves$w"
  done
done
