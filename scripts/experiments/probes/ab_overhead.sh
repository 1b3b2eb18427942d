#!/bin/bash
# Per-frame overhead A/B (frame wall time vs trace kernel): variants given as env assignments,
# each run twice, interleaved. Prints: variant frame_ms render_ms trace_ms Mrays/s.
# Usage (on the GPU box, from the repo root): scripts/ab_overhead.sh "SF_ORDER_ASYNC=1" "SF_ORDER_ASYNC=0" ...
set -e
OUT=gpurun_out/abo; mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --steps 200 --warmup 20 > $OUT/b.json
    python3 -c "import json,sys; j=json.load(open('$OUT/b.json')); print('$v', j['frame_ms'], j['kernel_ms'], j['roofline']['kernel_ms'], j['value'])"
  done
done
