#!/bin/bash
# round 6: the heavy-first order's rebuild period for whole 1080p frames (SF_ORDER_EVERY; default 64) against the
# driver's 20-step line, interleaved runs
set -o pipefail
O=gpurun_out/${TAG:-r6oe}; mkdir -p $O
for r in 1 2 3 4 5 6; do
  for ev in 64 256 1000000; do
    SF_ORDER_EVERY=$ev timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); p=d['pipeline']; print('every=$ev', d['ms_per_step'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', d['frame_latency_ms'], 'clk', d['roofline']['clock_mhz_live'], 'exact', d['check']['bit_exact'])" | tee -a $O/order_every.txt
  done
done
