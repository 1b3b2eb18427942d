#!/bin/bash
# Do the heavy-first order's kernels stall their slot's queue? A kernel trace of a bench run (order kernels' durations
# and the trace behind them), then 20-step lines for order rebuilds every 16th render (default), every 64th, never.
set -e
R=$PWD; OUT=$R/gpurun_out/r5order; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 $R/bench.py --steps 200 --warmup 30 --no-cpu-baseline --no-extras > $OUT/tr.log 2>&1
cd $R; python3 scripts/order_stall.py $(find $OUT/tr -name "*kernel_trace.csv") | tee $OUT/order_stall.txt; rm -rf $OUT/tr
for rep in 1 2 3 4 5; do
  for v in 16 64 off; do
    if [ $v = off ]; then E="SF_ORDER=0"; else E="SF_ORDER_EVERY=$v"; fi
    env $E timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $OUT/b.json 2>/dev/null
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('$v', 'frame', j['frame_ms'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', j['frame_latency_ms'], 'exact', j['check']['bit_exact'])"
  done
done | tee $OUT/ab20.txt
