#!/bin/bash
# Lone-frame latency with the drain polling the stream (SF_SPIN_US) against the blocking wait.
set -e
OUT=gpurun_out/r5spin; mkdir -p $OUT
for rep in 1 2; do for sp in 0 300; do
  SF_SPIN_US=$sp timeout -k 10 120 python3 -u scripts/lone_frame_timeline.py > $OUT/plain_$sp.txt 2>&1; echo "spin $sp: $(grep lone $OUT/plain_$sp.txt)"
done; done
for sp in 0 300; do
  SF_SPIN_US=$sp timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $OUT/b_$sp.json 2>/dev/null
  python3 -c "import json; j=json.loads(open('$OUT/b_$sp.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('spin $sp', 'frame', j['frame_ms'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', j['frame_latency_ms'], 'exact', j['check']['bit_exact'])"
done
