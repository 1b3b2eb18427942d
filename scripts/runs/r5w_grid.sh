#!/bin/bash
# The persistent grid's size for whole 1080p frames (3 frames in flight): all wave slots (default) vs fewer blocks.
set -e
mkdir -p gpurun_out/r5grid
REPS=3 timeout -k 10 1000 scripts/knob_sweep.sh r5grid "SF_NONE=0|" "SF_MAX_BLOCKS=6144|" "SF_MAX_BLOCKS=4096|" > gpurun_out/r5grid/sweep.txt 2>&1 || { tail -5 gpurun_out/r5grid/sweep.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5grid/sweep.txt
