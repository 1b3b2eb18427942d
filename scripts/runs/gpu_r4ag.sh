#!/bin/bash
# Round 4: the timed region's end without the redundant synchronize calls (the device synchronize covers the slot
# streams): the 20-step command x5 and the default line.
R=$PWD; OUT=$R/gpurun_out/r4ag; mkdir -p $OUT
for rep in 1 2 3 4 5; do
  timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $OUT/b20_$rep.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 7; }
  python3 -c "import json; j=json.loads(open('$OUT/b20_$rep.json').read().strip().split(chr(10))[-1]); print('steps20', j['frame_ms'], 'fill', j['pipeline']['fill_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'clk', j['roofline']['clock_mhz_live'], 'check', j['check']['bit_exact'])"
done
timeout -k 10 300 python3 -u bench.py > $OUT/b200.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 8; }
python3 -c "import json; j=json.loads(open('$OUT/b200.json').read().strip().split(chr(10))[-1]); print('default', j['frame_ms'], j['value'], 'fill', j['pipeline']['fill_ms'], 'clk', j['roofline']['clock_mhz_live'], 'traffic', j['roofline']['traffic'], 'check', j['check']['bit_exact'])"
