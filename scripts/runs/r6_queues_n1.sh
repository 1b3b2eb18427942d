#!/bin/bash
# round 6: the whole 1080p frame (N = 1, 3 in flight) with the runtime's 4 hardware queues against bench.py's 16,
# interleaved on one box: 200-step and 20-step lines
set -o pipefail
O=gpurun_out/${TAG:-r6qn}; mkdir -p $O
for r in 1 2 3 4; do
  for q in 0 16; do
    SF_HW_QUEUES=$q timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $O/b.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); p=d['pipeline']; print('sf_hw_queues=$q hwq', d['config'].get('hw_queues'), 'frame20', d['ms_per_step'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', d['frame_latency_ms'], 'clk', d['roofline']['clock_mhz_live'], 'exact', d['check']['bit_exact'])" | tee -a $O/n1.txt
  done
done
