#!/bin/bash
# Scheduling knobs against the current kernel (diagnostics): interleaved 200-step and 20-step bench lines per variant.
# Usage (GPU box, repo root): [REPS=2] scripts/knob_sweep.sh <tag> "<ENV=.. ENV=..>|<bench args>" ...
#   a variant is "ENV=v ... | extra bench args" (either side may be empty)
set -e
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    E=${v%%|*}; A=${v#*|}; [ "$A" = "$v" ] && A=""
    for st in "200 30" "20 5"; do
      S=${st% *}; W=${st#* }
      env $E timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --steps $S --warmup $W $A > $OUT/v$i.json 2> $OUT/v$i.err
      python3 -c "import json; j=json.loads(open('$OUT/v$i.json').read().strip().split(chr(10))[-1]); print('[$v] steps $S', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'lat', j['frame_latency_ms'], 'clk', j['roofline'].get('clock_mhz_live'))"
    done
  done
done
