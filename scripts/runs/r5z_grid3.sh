#!/bin/bash
set -e
mkdir -p gpurun_out/r5grid4
REPS=3 timeout -k 10 1100 scripts/knob_sweep.sh r5grid4 "SF_INFLIGHT_CAP=0 SF_MAX_BLOCKS=4096|" "SF_INFLIGHT_CAP=1|" "|" > gpurun_out/r5grid4/sweep.txt 2>&1 || { tail -5 gpurun_out/r5grid4/sweep.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5grid4/sweep.txt | grep "steps 200"
