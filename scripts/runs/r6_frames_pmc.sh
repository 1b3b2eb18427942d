#!/bin/bash
# round 6: PMC of one batch-8 launch of 1/8 shares (sf_trace_frames1) against the whole 1080p frame's launch
# (sf_trace_queue1): the same 32 400 tiles, ~2x the time -- instructions, waits or occupancy?
set -o pipefail
R=$PWD
O=$R/gpurun_out/${TAG:-r6fp}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in "batch --share 8 --configs 16:8" "full --configs 3:1"; do
  set -- $cfg; name=$1; shift
  for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
    n=$(echo $P | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $O/pmc_${name}_$n -o run --output-format csv -- python3 $R/scripts/frames_probe.py 1920 1080 0.25 --reps 1 --short 8 --long 24 "$@" > $O/pmc_${name}_$n.log 2>&1 || exit 1
  done
  python3 $R/scripts/pmc_summary.py $O/pmc_${name}_*/ > $O/pmc_$name.txt 2>&1
  grep -A18 "sf_trace_frames1 \|sf_trace_queue1 " $O/pmc_$name.txt | head -40
done
