#!/bin/bash
# A/B of env variants on one BASELINE config: scripts/ab_config.sh "<bench args>" "ENV=.." ...
# Prints: variant frame_ms trace_ms Mrays/s (each variant twice, interleaved).
set -e
ARGS=$1; shift
OUT=gpurun_out/abc; mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras $ARGS > $OUT/b.json
    python3 -c "import json; j=json.load(open('$OUT/b.json')); print('$v', j['frame_ms'], j['roofline']['kernel_ms'], j['value'])"
  done
done
