#!/bin/bash
# Round 4: in-wave tie re-trace (no fixup launch when the levels are proven), fixed tests, long-loop placement; the
# order-knob A/B on the driver's 20-step command.
R=$PWD; OUT=$R/gpurun_out/r4b; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head -20
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err || { tail -20 $OUT/bench20.err; exit 4; }
python3 -c "
import json
j = json.loads(open('$OUT/bench20.json').read().strip().splitlines()[-1])
print('bench20', j['value'], j['ms_per_step'], 'lat', j['frame_latency_ms'], 'pipe', {k: v for k, v in j['pipeline'].items() if k != 'note'}, 'check', j['check']['bit_exact'], 'frac', j['roofline']['frac'], 'frameless', j['frameless'])
"
bash scripts/runs/order_ab.sh r4b/ab 2 || exit 5
for steps in 20 200; do
  for v in 1 0; do
    SF_TIE_INLINE=$v timeout -k 10 120 python3 -u bench.py --steps $steps --warmup 5 --no-cpu-baseline --no-extras > $OUT/tie$v.json 2>/dev/null || exit 6
    python3 -c "import json; j=json.loads(open('$OUT/tie$v.json').read().strip().splitlines()[-1]); print('tie_inline=$v steps $steps', j['ms_per_step'], j['pipeline']['steady_frame_ms'], j['frame_latency_ms'])"
  done
done
exit $rc
