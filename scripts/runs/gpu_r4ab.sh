#!/bin/bash
# Round 4: the driver's 20-step command, 8 runs with per-frame enqueue times (SF_BENCH_ENQ_TRACE=1): where a slow
# run loses its time.
R=$PWD; OUT=$R/gpurun_out/r4ab; mkdir -p $OUT
for rep in 1 2 3 4 5 6 7 8; do
  SF_BENCH_ENQ_TRACE=1 timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $OUT/b$rep.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 7; }
  python3 - $OUT/b$rep.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
tr = j.get("enqueue_trace_us", [[]])[0]
gaps = [round(b - a, 1) for a, b in zip([0.0] + tr[:-1], tr)]
print("frame", j["frame_ms"], "fill", j["pipeline"]["fill_ms"], "clk", j["roofline"]["clock_mhz_live"], "enq gaps us", gaps)
PY
done
