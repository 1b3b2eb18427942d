#!/bin/bash
# Round 4: the 20-step command's run-to-run spread against the tile-order schedule: default (heavy-first order
# rebuilt every 16th render), SF_ORDER_EVERY=4, SF_ORDER=0 (row-major), interleaved x5.
R=$PWD; OUT=$R/gpurun_out/r4ac; mkdir -p $OUT
for rep in 1 2 3 4 5; do
  for v in "def SF_NOP=1" "every4 SF_ORDER_EVERY=4" "order0 SF_ORDER=0"; do
    set -- $v; name=$1; shift
    env "$@" timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 7; }
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$name', 'frame', j['frame_ms'], 'fill', j['pipeline']['fill_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'lat', j['frame_latency_ms'], 'clk', j['roofline']['clock_mhz_live'])"
  done
done
