# Frames in flight for the whole frame (N=1 bench) with the round-3 defaults: slots 3 vs 4 vs 5, interleaved.
R=$PWD; OUT=$R/gpurun_out/r3ap; mkdir -p $OUT
for rep in 1 2; do
  for s in 3 4 5; do
    timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --slots $s > $OUT/b.json 2>$OUT/b.err || exit 1
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('slots $s', 'frame', j['frame_ms'], 'Mrays', j['value'], 'clk', j['roofline'].get('clock_mhz_live'))"
  done
done
