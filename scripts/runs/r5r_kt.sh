#!/bin/bash
# The driver's 20-step line with 8 kernel-timing samples (every 2nd frame per slot) vs 3 (one per slot).
set -e
R=$PWD; OUT=$R/gpurun_out/r5kt; mkdir -p $OUT
for rep in 1 2 3 4; do
  for kt in 8 3; do
    SF_BENCH_KT_MIN=$kt timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/b_$kt.json 2>/dev/null
    python3 -c "import json; j=json.loads(open('$OUT/b_$kt.json').read().strip().split(chr(10))[-1]); print('kt $kt', 'ms', j['ms_per_step'], 'samples', j.get('kernel_samples') or j['roofline'].get('kernel_samples'), 'fill', j['pipeline'].get('fill_ms'), 'clk', j['roofline'].get('clock_mhz_live'))"
  done
done 2>&1 | tee $OUT/kt.txt
