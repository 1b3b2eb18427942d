#!/bin/bash
# Round 4, first GPU call on the reworked gather (4-B index slabs, receive/unpack stream) and bench line:
# full -m gpu suite, smoke, the driver's bench command and the default one, a rows-mode rehearsal under a kernel
# trace (unpack beside member 0's trace), and the spawned 2-rank rehearsal (bench.py --gpus 2 without a launcher).
# Each GPU step has its own limit; a crash or time limit ends the script.
R=$PWD; OUT=$R/gpurun_out/r4a; mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'sphereflake-raytracer_amd'); import sphereflake_amd as sf; print(sf.build_info())" > $OUT/build_info.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
cat $OUT/smoke.log
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err || { tail -20 $OUT/bench20.err; exit 4; }
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
python3 -c "
import json
for f in ('bench20', 'bench'):
    j = json.loads(open('$OUT/%s.json' % f).read().strip().splitlines()[-1])
    print(f, j['value'], j['ms_per_step'], 'lat', j['frame_latency_ms'], 'pipe', j.get('pipeline'), 'check', j.get('check', {}).get('bit_exact'), 'frac', j['roofline']['frac'])
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rows8 -o run --output-format csv -- python3 $R/bench.py --mode rows --gpus 8 --steps 60 --warmup 5 --no-cpu-baseline > $OUT/rows8.log 2>&1 || { tail -20 $OUT/rows8.log; exit 5; }
grep '^{' $OUT/rows8.log | tail -1
python3 $R/scripts/unpack_overlap.py $(find $OUT/rows8 -name "*kernel_trace.csv") | tee $OUT/rows8_overlap.txt
cd $R
timeout -k 10 300 python3 -u bench.py --gpus 2 --rehearse --steps 40 --warmup 5 > $OUT/spawn2.json 2> $OUT/spawn2.err || { tail -20 $OUT/spawn2.err; exit 6; }
tail -1 $OUT/spawn2.json | cut -c1-600
exit $rc
