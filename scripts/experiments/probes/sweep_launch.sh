#!/bin/bash
# Launch-shape sweep (waves per workgroup x LDS levels) of the wave kernel at the bench config.
# Run on the GPU box from the repo root; one bench process per point (env knobs are read at context creation).
set -e
mkdir -p gpurun_out/sweep
for W in 1 2 4; do
  for L in 9 12; do
    SF_TRACE_WAVES=$W SF_LEVELS=$L timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/sweep/w${W}_l${L}.json 2> gpurun_out/sweep/w${W}_l${L}.err
    echo "waves=$W levels=$L $(python3 -c "import json;d=json.loads(open('gpurun_out/sweep/w${W}_l${L}.json').readlines()[-1]);print(d['value'],d['kernel_ms'])")"
  done
done
