#!/bin/bash
# round 6: frames in flight x hardware queues over the whole share curve (N = 1, 2, 4, 8; 1080p and 4K), and the
# bench's own N = 1 lines with GPU_MAX_HW_QUEUES 4 vs 16
set -o pipefail
O=gpurun_out/${TAG:-r6qc}; mkdir -p $O
for q in 4 16; do
  echo "hwq $q 1080p" | tee -a $O/curve.txt
  GPU_MAX_HW_QUEUES=$q PROBE_N=1,2,4,8 PROBE_SLOTS=3,4,6,8 timeout -k 10 400 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | tee -a $O/curve.txt || exit 1
done
echo "hwq 16 4K" | tee -a $O/curve.txt
GPU_MAX_HW_QUEUES=16 PROBE_N=1,8 PROBE_SLOTS=3,4,6 timeout -k 10 400 python3 -u scripts/share_probe.py 3840 2160 0.22 2>&1 | grep -v amdgpu.ids | tee -a $O/curve.txt || exit 1
for r in 1 2; do
  for q in 4 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $O/b.json 2>/dev/null || exit 1
    python3 -c "import json; j=json.loads(open('$O/b.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('hwq $q', 'frame20', j['ms_per_step'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', j['frame_latency_ms'], 'exact', j['check']['bit_exact'])" | tee -a $O/bench.txt
  done
done
