#!/bin/bash
# Round 5: the one-barrier mt19937 twist: frame-less parity tests, then the draws alone under a kernel trace.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5l
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -k "progressive or mt or frameless or initialize" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
SF_PROG_PREFETCH=0 PROG_BATCHES=262144 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/frameless_alone -o run --output-format csv -- python3 $R/scripts/prog_bench.py > $OUT/frameless_alone.log 2>&1
grep -v amdgpu $OUT/frameless_alone.log | tail -3
cat $(find $OUT/frameless_alone -name "*kernel_stats.csv") | grep -i "mt_\|Name"
