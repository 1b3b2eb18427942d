#!/bin/bash
# A/B of the heavy-first tile order's knobs on the driver's bench command (20 steps) and the default (200): frame
# period, pipeline fill (drain), lone-frame latency. Interleaved reps. Usage: order_ab.sh <tag> [reps]
R=$PWD; OUT=$R/gpurun_out/${1:-order_ab}; mkdir -p $OUT; REPS=${2:-2}
run() {  # run <name> <steps> <env...>
  local name=$1 steps=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --steps $steps --warmup 5 --no-cpu-baseline --no-extras > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; return 1; }
  python3 -c "
import json; j=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); p=j.get('pipeline',{})
print('%-10s steps %3d frame %.4f steady %.4f fill %.4f lat %.4f fixed %.4f check %s' % ('$name', $steps, j['ms_per_step'], p.get('steady_frame_ms',0), p.get('fill_ms',0), j['frame_latency_ms'], j['fixed_camera']['frame_ms'], j.get('check',{}).get('bit_exact')))"
}
for rep in $(seq $REPS); do
  for steps in 20 200; do
    run base_$steps $steps SF_NOP=1 || exit 1
    run ord_$steps $steps SF_ORDER=1 || exit 1
    run ord16r_$steps $steps SF_ORDER=1 SF_ORDER_EVERY=16 SF_ORDER_RECORD=0 || exit 1
    run ord4r_$steps $steps SF_ORDER=1 SF_ORDER_EVERY=4 SF_ORDER_RECORD=0 || exit 1
    run ord16m_$steps $steps SF_ORDER=1 SF_ORDER_EVERY=16 SF_ORDER_RECORD=0 SF_SPLIT_BUCKETS=model || exit 1
  done
done
