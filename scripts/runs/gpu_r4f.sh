#!/bin/bash
# Round 4: synchronize without the second round trip, SSAO taps fetched together; full suite, bench (driver's
# command and default), lone-frame probe, post probe, split-bucket A/B on the 20-step command.
R=$PWD; OUT=$R/gpurun_out/r4f; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head -20
SF_FLAGS=0x20 timeout -k 10 120 python3 -u scripts/latency_probe.py > $OUT/latency.txt 2>&1 || { tail -5 $OUT/latency.txt; exit 3; }
grep frame $OUT/latency.txt | cut -c1-200
timeout -k 10 120 python3 -u scripts/post_probe.py > $OUT/post.txt 2>&1 || { tail -5 $OUT/post.txt; exit 4; }
cat $OUT/post.txt
run() {  # run <name> <steps> <env...>
  local name=$1 steps=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --steps $steps --warmup 5 --no-cpu-baseline --no-extras > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; return 1; }
  python3 -c "
import json; j=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); p=j.get('pipeline',{})
print('%-10s steps %3d frame %.4f steady %.4f fill %.4f lat %.4f fixed %.4f check %s' % ('$name', $steps, j['ms_per_step'], p.get('steady_frame_ms',0), p.get('fill_ms',0), j['frame_latency_ms'], j['fixed_camera']['frame_ms'], j.get('check',{}).get('bit_exact')))"
}
for rep in 1 2; do
  for steps in 20 200; do
    run model_$steps $steps SF_NOP=1 || exit 5
    run top1_$steps $steps SF_SPLIT_BUCKETS=1 || exit 5
    run top2_$steps $steps SF_SPLIT_BUCKETS=2 || exit 5
  done
done
exit $rc
