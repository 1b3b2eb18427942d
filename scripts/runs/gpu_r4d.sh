#!/bin/bash
# Round 4: the new defaults (order on frames over twice the grid, prefetch stream priority, XCD-aware post tiles,
# hoisted post reciprocals): full -m gpu suite, smoke, the driver's bench command and the default one, the post
# probe under a kernel trace + FETCH_SIZE, the BASELINE configs.
R=$PWD; OUT=$R/gpurun_out/r4d; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head -20
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
for rep in 1 2; do
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20_$rep.json 2> $OUT/bench20_$rep.err || { tail -20 $OUT/bench20_$rep.err; exit 4; }
  timeout -k 10 400 python3 -u bench.py > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || { tail -20 $OUT/bench_$rep.err; exit 4; }
done
python3 -c "
import json
for f in ('bench20_1', 'bench_1', 'bench20_2', 'bench_2'):
    j = json.loads(open('$OUT/%s.json' % f).read().strip().splitlines()[-1])
    print(f, j['value'], j['ms_per_step'], 'lat', j['frame_latency_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'check', j['check']['bit_exact'], 'frac', j['roofline']['frac'], 'post', j['post']['fused_ms'], 'fl', j['frameless']['avx']['ms_per_batch'], j['frameless']['sse']['ms_per_batch'], 'c4', j['configs']['c4']['frame_ms'])
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/post -o run --output-format csv -- python3 $R/scripts/post_probe.py > $OUT/post.log 2>&1 || { tail -5 $OUT/post.log; exit 5; }
grep post $OUT/post.log; grep -E "sf_post" $(find $OUT/post -name "*kernel_stats.csv") | cut -d, -f1-4
POST_REPS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/post_pm1 -o run --output-format csv -- python3 $R/scripts/post_probe.py > $OUT/post_pm1.log 2>&1 || echo "pmc failed"
cd $R
bash scripts/configs_bench.sh r4d/cfg > $OUT/configs.log 2>&1 || { tail -5 $OUT/configs.log; exit 7; }
grep -E "^c[0-9]|batch" $OUT/configs.log
exit $rc
