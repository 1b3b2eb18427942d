#!/bin/bash
# The round's evidence on the GPU box for the library built in-tree: the full -m gpu suite, smoke(), the
# default bench line, a rocprofv3 kernel-trace profile of the bench, the PMC passes (recorded with the library
# build in pmc_traffic.json, collected before the bench so that its line carries them) and, optionally, an LDS A/B of variant builds. Each GPU step has its own limit;
# a test failure (pytest 1) still lets the rest run, a time limit or crash ends the script.
# Usage (on the box, repo root): scripts/round_profile.sh <tag> [variant.so ...]
TAG=${1:-r3}; shift || true
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cp -f BUILD_SHA $OUT/ 2>/dev/null || true
python3 -c "import sys; sys.path.insert(0, 'sphereflake-raytracer_amd'); import sphereflake_amd as sf; print(sf.build_info())" > $OUT/build_info.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
cat $OUT/smoke.log
# the PMC passes first, their summary in place as profiles/pmc_traffic.json (this box's copy): the bench lines
# below then carry `traffic` and `valu` for this very library build
scripts/prof_pmc.sh $TAG/pmc || exit 6
python3 scripts/pmc_summary.py --json $OUT/pmc_traffic.json --config "1920x1080 K=0.25 moving" $OUT/pmc/*/ > $OUT/pmc_summary.txt
head -40 $OUT/pmc_summary.txt
cp -f $OUT/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
tail -1 $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 5; }
cat $(find $OUT/stats -name "*kernel_stats.csv") | head -12
grep '^{' $OUT/stats.log | tail -1 > $OUT/bench_under_rocprof.json
# timed loop of the default bench: 1 code-object warm-up + 1 first render + 30 warmup + the settle frames,
# then 200 timed dispatches
SKIP=$(python3 -c "import json; print(32 + json.load(open('$OUT/bench_under_rocprof.json'))['settle']['frames'])")
python3 $R/scripts/trace_avg.py $(find $OUT/stats -name "*kernel_trace.csv") sf_trace_queue1 200 $SKIP | tee $OUT/trace_avg.txt
cd $R
if [ $# -gt 0 ]; then REPS=0 PMC=1 scripts/lib_ab.sh $TAG/lds "" sphereflake-raytracer_amd/build/libsphereflake_hip.so "$@"; fi
exit $rc
