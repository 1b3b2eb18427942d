#!/bin/bash
# Round 4: the bench after the clock fix (kernel timing switched on before the warm-up) and the frames-in-flight rule.
R=$PWD; OUT=$R/gpurun_out/r4o; mkdir -p $OUT
show() { python3 -c "import json; j=json.loads(open('$1').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('$2', 'frame', j['frame_ms'], 'clk', j['roofline']['clock_mhz_live'], 'long', p['long_frame_ms'], 'clk', p['long_clock_mhz_live'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', j['frame_latency_ms'], 'slots', j['config']['slots'], 'check', j['check']['bit_exact'])"; }
for rep in 1 2; do
  timeout -k 10 150 python3 -u bench.py --no-cpu-baseline > $OUT/b200_$rep.json 2> $OUT/b200_$rep.err || { tail -3 $OUT/b200_$rep.err; exit 7; }
  show $OUT/b200_$rep.json "default"
  timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/b20_$rep.json 2> $OUT/b20_$rep.err || { tail -3 $OUT/b20_$rep.err; exit 7; }
  show $OUT/b20_$rep.json "steps20"
  timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --width 640 --height 360 --K 1.0 > $OUT/c1_$rep.json 2> $OUT/c1_$rep.err || { tail -3 $OUT/c1_$rep.err; exit 7; }
  show $OUT/c1_$rep.json "c1"
done
