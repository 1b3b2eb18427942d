#!/bin/bash
# Round 4: the driver's 20-step command against the number of kernel-timing samples in its timed loop (HIP events
# around the sampled trace launches): 8 (default) vs 1 per slot, interleaved.
R=$PWD; OUT=$R/gpurun_out/r4aa; mkdir -p $OUT
for rep in 1 2 3; do
  for k in 8 1; do
    SF_BENCH_KSAMPLES=$k timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 7; }
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('ksamples $k', 'frame', j['frame_ms'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'clk', j['roofline'].get('clock_mhz_live'), 'samples', j['roofline'].get('kernel_samples'))"
  done
done
