#!/bin/bash
# Round 4: the live clock of the bench's timed loop and of its long loop, 3 vs 4 frames in flight.
R=$PWD; OUT=$R/gpurun_out/r4l; mkdir -p $OUT
for s in 3 4 3 4; do
  timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --slots $s > $OUT/b_s$s.json 2> $OUT/b_s$s.err || { tail -3 $OUT/b_s$s.err; exit 7; }
  python3 -c "import json; j=json.loads(open('$OUT/b_s$s.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('slots $s', 'frame', j['frame_ms'], 'clk', j['roofline']['clock_mhz_live'], 'long', p['long_frame_ms'], 'clk', p['long_clock_mhz_live'], 'steady', p['steady_frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'settle', j['settle'])"
done
