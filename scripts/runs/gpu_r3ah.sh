# Queues per XCD x tile-order cadence on the round-end kernel (1080p and 4K), interleaved, 2 reps.
R=$PWD; OUT=$R/gpurun_out/r3ah; mkdir -p $OUT
for rep in 1 2; do
for kv in "SF_NONE=0" "SF_QUEUES_PER_XCD=4 SF_ORDER_EVERY=2" "SF_QUEUES_PER_XCD=4 SF_ORDER_EVERY=3" "SF_QUEUES_PER_XCD=4 SF_ORDER_EVERY=4" "SF_QUEUES_PER_XCD=4 SF_ORDER=0" "SF_QUEUES_PER_XCD=2 SF_ORDER_EVERY=3"; do
  env $kv timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/k.json 2>/dev/null || exit 6
  python3 -c "import json; j=json.loads(open('$OUT/k.json').read().strip().split(chr(10))[-1]); print('$kv'.replace(' ', '+'), '1080p frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'lat', j['frame_latency_ms'])"
  env $kv timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --width 3840 --height 2160 --K 0.22 --steps 100 > $OUT/k.json 2>/dev/null || exit 7
  python3 -c "import json; j=json.loads(open('$OUT/k.json').read().strip().split(chr(10))[-1]); print('$kv'.replace(' ', '+'), '4K frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'])"
done
done
