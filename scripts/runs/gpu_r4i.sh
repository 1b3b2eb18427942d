#!/bin/bash
# Round 4: a member's share at 3-5 frames in flight in a torch process (as the bench's), 4 / 8 hardware queues.
R=$PWD; OUT=$R/gpurun_out/r4i; mkdir -p $OUT
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q PROBE_TORCH=1 PROBE_STEPS=600 PROBE_N=1,2,4,8 PROBE_SLOTS=3,4,5 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/share_q$q.txt 2>&1 || { tail -3 $OUT/share_q$q.txt; exit 6; }
  echo "== GPU_MAX_HW_QUEUES=$q"; grep slots $OUT/share_q$q.txt
done
for s in 3 4; do
  timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 20 --slots $s --no-check --no-cpu-baseline > $OUT/bench_s$s.json 2> $OUT/bench_s$s.err || { tail -3 $OUT/bench_s$s.err; exit 7; }
  python3 -c "import json; d=json.load(open('$OUT/bench_s$s.json')); print('slots $s', d['ms_per_step'], d['roofline']['clock_mhz_live'], d['pipeline']['steady_frame_ms'])"
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 20 --slots $s --no-check --no-cpu-baseline > $OUT/bench_s${s}_q8.json 2> $OUT/bench_s${s}_q8.err || { tail -3 $OUT/bench_s${s}_q8.err; exit 7; }
  python3 -c "import json; d=json.load(open('$OUT/bench_s${s}_q8.json')); print('slots $s q8', d['ms_per_step'], d['roofline']['clock_mhz_live'], d['pipeline']['steady_frame_ms'])"
done
