#!/bin/bash
# round 6: the bench's projected member-share leg with the kernel-timing events off (default) and on
set -o pipefail
O=gpurun_out/${TAG:-r6st}; mkdir -p $O
for r in 1 2; do
  for t in 0 1; do
    SF_BENCH_SHARES_TIMING=$t timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); m=d['member_shares']; print('timing $t', d['ms_per_step'], ' '.join(f\"{k}: {m[k]['steady_ms']} ({m[k]['speedup']}x, {m[k]['slots']} slots)\" for k in ('n2','n4','n8')))" | tee -a $O/shares_timing.txt
  done
done
