#!/bin/bash
# A/B sweep of launch/feature knobs at the bench config (one bench process per point; the env knobs
# are read at context creation). Usage (GPU box, repo root): scripts/sweep.sh <tag> "<ENV=.. ENV=..>" ...
set -e
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/p$i.json 2> gpurun_out/$TAG/p$i.err
  echo "$cfg => $(python3 -c "import json;d=json.loads(open('gpurun_out/$TAG/p$i.json').readlines()[-1]);print(d['value'],d['kernel_ms'])")"
done
