#!/bin/bash
# Kernel stats of a short default bench under rocprofv3 (kernel trace only). Usage: scripts/prof_quick.sh <tag>
set -e
R=$PWD; OUT=$R/gpurun_out/${1:-pq}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras > $OUT/bench.log 2>&1
grep -h 'sf_' $(find $OUT -name "*kernel_stats.csv")
grep '^{' $OUT/bench.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['frame_ms'], j['value'])"
