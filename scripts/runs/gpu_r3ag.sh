# Scheduling knobs on the round-end kernel, interleaved, 2 reps each (second sweep: queues per XCD combinations).
R=$PWD; OUT=$R/gpurun_out/r3ag; mkdir -p $OUT
for rep in 1 2; do
for kv in "SF_NONE=0" "SF_QUEUES_PER_XCD=2" "SF_QUEUES_PER_XCD=4" "SF_QUEUES_PER_XCD=2 SF_ORDER_EVERY=2" "SF_QUEUES_PER_XCD=4 SF_ORDER_EVERY=2" "SF_QUEUES_PER_XCD=2 SF_TRACE_WAVES=4" "SF_QUEUES_PER_XCD=4 SF_TRACE_WAVES=4"; do
  env $kv timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/k.json 2>/dev/null || exit 6
  python3 -c "import json; j=json.loads(open('$OUT/k.json').read().strip().split(chr(10))[-1]); print('$kv'.replace(' ', '+'), 'frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'lat', j['frame_latency_ms'], 'clk', j['roofline']['clock_mhz_live'])"
done
done
