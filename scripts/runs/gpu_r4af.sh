#!/bin/bash
# Round 4: kernel traces of the 20-step command, 5 runs: what a slow run's timed loop does differently on the GPU.
R=$PWD; OUT=$R/gpurun_out/r4af; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3 4 5; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/t$rep -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $OUT/b$rep.log 2>&1 || { tail -5 $OUT/b$rep.log; exit 5; }
  grep '^{' $OUT/b$rep.log | tail -1 > $OUT/b$rep.json
  python3 $R/scripts/loop_trace.py $(find $OUT/t$rep -name "*kernel_trace.csv") $OUT/b$rep.json 5 > $OUT/loop$rep.txt 2>&1
  head -1 $OUT/loop$rep.txt
done
