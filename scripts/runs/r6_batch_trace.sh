#!/bin/bash
# round 6: kernel trace of 8-frame share launches (16 slots, 16 queues): slow vs fast loops
set -o pipefail
R=$PWD
O=$R/gpurun_out/${TAG:-r6btr}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/scripts/frames_probe.py 1920 1080 0.25 --share 8 --reps 6 --configs 16:8 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt | tail -2
python3 $R/scripts/batch_trace_summary.py $(find $O/trace -name "*kernel_trace.csv") | tee $O/summary.txt
