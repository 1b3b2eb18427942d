#!/bin/bash
# Round 4: frames in flight 3 vs 4 on the whole-frame configs (640x360, 1280x720, 1080p), interleaved.
R=$PWD; OUT=$R/gpurun_out/r4j; mkdir -p $OUT
for rep in 1 2; do
for cfg in "c1 640 360 1.0" "c2 1280 720 0.8" "c3 1920 1080 0.25"; do
  set -- $cfg
  for s in 3 4; do
    timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --width $2 --height $3 --K $4 --slots $s > $OUT/bench_$1_s${s}_$rep.json 2> $OUT/bench_$1_s${s}_$rep.err || { tail -3 $OUT/bench_$1_s${s}_$rep.err; exit 7; }
    python3 -c "import json; j=json.loads(open('$OUT/bench_$1_s${s}_$rep.json').read().strip().split(chr(10))[-1]); print('$1 slots $s', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'lat', j['frame_latency_ms'], 'clk', j['roofline']['clock_mhz_live'], 'check', j['check']['bit_exact'])"
  done
done
done
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --gpus 2 --rehearse > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { tail -5 $OUT/rehearse2.err; exit 8; }
python3 -c "import json; j=json.loads(open('$OUT/rehearse2.json').read().strip().split(chr(10))[-1]); print('rehearse2', j['value'], j['config']['slots'], j['check']['bit_exact'])"
