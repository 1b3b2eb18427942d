#!/bin/bash
# One GPU-box pass: GPU parity tests, the default bench line, a kernel-trace profile of the bench,
# and the PMC passes. Every GPU step has its own time limit; the script stops at the first failure.
# Usage (on the box, from the repo root): scripts/round_gpu.sh <tag>
set -e
TAG=${1:-r1}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -3 $OUT/pytest_gpu.log
scripts/prof_pmc.sh $TAG/pmc
python3 scripts/pmc_summary.py --json $OUT/pmc_traffic.json --config "1920x1080 K=0.25 moving" $OUT/pmc/*/ > $OUT/pmc_summary.txt
cp $OUT/pmc_traffic.json $R/profiles/pmc_traffic.json
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras > $OUT/stats.log 2>&1
cat $(find $OUT/stats -name "*kernel_stats.csv")
python3 $R/scripts/trace_avg.py $(find $OUT/stats -name "*kernel_trace.csv") sf_trace_queue2 200 32 | tee $OUT/trace_avg.txt
grep '^{' $OUT/stats.log | tail -1
