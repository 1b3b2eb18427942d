#!/bin/bash
# A/B of subtree donation variants: GPU parity of the donation test, then bench lines per variant at c3
# and c1 (each twice, interleaved). Usage (on the box, repo root): scripts/ab_pair.sh <tag> "ENV=.." ...
set -e
OUT=gpurun_out/${1:-abp}; shift; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "donation" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in "" "--width 640 --height 360 --K 1.0"; do
  for rep in 1 2; do
    for v in "$@"; do
      env $v timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --steps 200 --warmup 30 $cfg > $OUT/b.json
      python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$cfg' or 'c3', '$v', j['frame_ms'], j['roofline']['kernel_ms'], j['value'], j['fixed_camera']['frame_ms'] if j.get('fixed_camera') else None, j['first_render_ms'])"
    done
  done
done
