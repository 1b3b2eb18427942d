#!/bin/bash
# round 6: with the contexts' own queues, the multi-frame batches of 1/8 shares (bench --batch 8) and the torch-free
# share probe
set -o pipefail
O=gpurun_out/${TAG:-r6cmb}; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --batch 8 > $O/b_batch.json 2> $O/b_batch.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_batch.json').read().strip().splitlines()[-1]); m=d['member_shares']; print('batch8', d['ms_per_step'], d['config'].get('frames_per_launch'), ' '.join(f\"{k}: {m[k]['steady_ms']} ({m[k]['speedup']}x, {m[k]['slots']} slots, {m[k]['frames_per_launch']}/launch)\" for k in ('n2','n4','n8')))" | tee -a $O/batches.txt
done
timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | tee -a $O/batches.txt
