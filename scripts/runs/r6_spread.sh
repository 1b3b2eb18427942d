#!/bin/bash
# round 6: the static first units spread over the first-dispatched waves (SF_SPREAD = stride, A/B): parity with the
# env set, the 1080p share over 8, and the whole 1080p frame (bench lines: steady period, 20-step line, lone frame)
set -o pipefail
O=gpurun_out/${TAG:-r6sp}; mkdir -p $O
SF_SPREAD=257 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_views.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_spread.txt 2>&1 || { tail -30 $O/pytest_spread.txt; exit 1; }
tail -1 $O/pytest_spread.txt
for r in 1 2; do
  for S in 0 37 127 257 1031; do
    echo -n "spread $S: " | tee -a $O/share.txt
    SF_SPREAD=$S PROBE_N=8 timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | sed 's/.*\]: //' | tee -a $O/share.txt || exit 1
  done
done
for r in 1 2; do
  for S in 0 257 1031; do
    SF_SPREAD=$S timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $O/b.json 2>/dev/null || exit 1
    python3 -c "import json; j=json.loads(open('$O/b.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('spread $S', 'frame20', j['ms_per_step'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', j['frame_latency_ms'], 'exact', j['check']['bit_exact'])" | tee -a $O/bench.txt
  done
done
