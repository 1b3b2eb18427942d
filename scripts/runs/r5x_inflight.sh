#!/bin/bash
# Whole frames beside frames in flight on half the grid (sf_dist): GPU suite, bench lines and lone frames, on/off.
set -e
R=$PWD; OUT=$R/gpurun_out/r5infl; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
REPS=4 timeout -k 10 1000 scripts/knob_sweep.sh r5infl "SF_INFLIGHT_CAP=0|" "SF_INFLIGHT_CAP=1|" > $OUT/sweep.txt 2>&1 || { tail -5 $OUT/sweep.txt; exit 1; }
grep -v amdgpu.ids $OUT/sweep.txt
for rep in 1 2; do for q in 0 1; do
  echo -n "cap$q "; SF_INFLIGHT_CAP=$q timeout -k 10 120 python3 -u scripts/lone_latency.py 300 2>&1 | grep "lone frame"
done; done
