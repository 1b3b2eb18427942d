#!/bin/bash
# A/B bench lines of env variants (each twice, interleaved) on a config.
# Usage (on the box, repo root): scripts/ab_bench.sh <tag> "<bench args>" "ENV=.." ...
set -e
OUT=gpurun_out/${1:-abb}; shift; ARGS=$1; shift; mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --steps 200 --warmup 30 $ARGS > $OUT/b.json
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('${ARGS:-c3}', '$v', 'frame', j['frame_ms'], 'trace', j['roofline']['kernel_ms'], 'Mrays', j['value'], 'fixed', j['fixed_camera']['frame_ms'] if j.get('fixed_camera') else None)"
  done
done
