#!/bin/bash
# round 6: another box's sample of the bench lines for the current library (the default line + three driver-shaped
# 20-step lines); usage: r6_bench_sample.sh <tag>
set -e
OUT=gpurun_out/${1:-r6bs}; mkdir -p $OUT
sha256sum sphereflake-raytracer_amd/build/libsphereflake_hip.so > $OUT/lib_sha256.txt
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $OUT/bench20_$i.json 2> $OUT/bench20_$i.err
done
for f in $OUT/bench.json $OUT/bench20_1.json $OUT/bench20_2.json $OUT/bench20_3.json; do
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); p=d['pipeline']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', d['frame_latency_ms'], 'clk', d['roofline']['clock_mhz_live'], 'frac', d['roofline']['frac'], 'exact', d['check']['bit_exact'], 'n8', d['member_shares']['n8']['steady_ms'])" | tee -a $OUT/summary.txt
done
