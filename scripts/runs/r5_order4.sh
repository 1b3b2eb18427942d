#!/bin/bash
# Order rebuild in one-wave workgroups: GPU suite, stall analysis, 20-step lines at rebuild every 16th / 64th render.
set -e
R=$PWD; OUT=$R/gpurun_out/r5order4; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
SF_ORDER_EVERY=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 $R/bench.py --steps 200 --warmup 30 --no-cpu-baseline --no-extras > $OUT/tr.log 2>&1
cd $R; python3 scripts/order_stall.py $(find $OUT/tr -name "*kernel_trace.csv") | tee $OUT/order_stall.txt; rm -rf $OUT/tr
for rep in 1 2 3 4 5; do
  for v in 16 64; do
    SF_ORDER_EVERY=$v timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $OUT/b.json 2>/dev/null
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('$v', 'frame', j['frame_ms'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', j['frame_latency_ms'], 'exact', j['check']['bit_exact'])"
  done
done | tee $OUT/ab20.txt
