#!/bin/bash
# Round 4: scheduling knobs with the one-wave kernel (1080p default bench, interleaved x2): queue words per XCD,
# graded priority buckets, order rebuild period.
R=$PWD; OUT=$R/gpurun_out/r4ai; mkdir -p $OUT
for rep in 1 2; do
  for v in "def SF_NOP=1" "qpx2 SF_QUEUES_PER_XCD=2" "qpx1 SF_QUEUES_PER_XCD=1" "prio0 SF_PRIO_BUCKETS=0" "prio12 SF_PRIO_BUCKETS=12" "every8 SF_ORDER_EVERY=8" "every32 SF_ORDER_EVERY=32" "order0 SF_ORDER=0"; do
    set -- $v; name=$1; shift
    env "$@" timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 7; }
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$name', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'lat', j['frame_latency_ms'], 'clk', j['roofline']['clock_mhz_live'], 'check', j['check']['bit_exact'])"
  done
done
