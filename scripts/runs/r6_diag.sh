#!/bin/bash
# Round-6 diagnosis of the multi-frame kernel's throughput: the same frames one per launch through either kernel
# (SF_FRAMES_ONE=1: sf_trace_frames1 with one frame), batches with and without the interleaved heads, and one PMC
# pass of the SQ counters per configuration.
set -o pipefail
OUT=$PWD/gpurun_out/${1:-r6d}
mkdir -p $OUT
export TMPDIR=/tmp
SF_FRAMES_ONE=1 timeout -k 10 200 python -u scripts/frames_probe.py 1920 1080 0.25 --configs "3:1,3:-1,4:4" > $OUT/probe_one.txt 2>&1
rc=$?; cat $OUT/probe_one.txt; [ $rc -ne 0 ] && exit $rc
SF_FRAMES_HEAVY=0 timeout -k 10 200 python -u scripts/frames_probe.py 1920 1080 0.25 --configs "4:4,8:8" > $OUT/probe_heavy0.txt 2>&1
rc=$?; cat $OUT/probe_heavy0.txt; [ $rc -ne 0 ] && exit $rc
R=$PWD
cd /tmp
for cfg in "3:1" "3:-1" "4:4"; do
  tag=$(echo $cfg | tr ':-' '_m')
  SF_FRAMES_ONE=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $OUT/pmc_$tag -o run --output-format csv -- python3 $R/scripts/frames_probe.py 1920 1080 0.25 --configs "$cfg" --reps 1 --short 20 --long 40 > $OUT/pmc_$tag.log 2>&1 || exit 7
done
cd $R
python3 scripts/pmc_summary.py $OUT/pmc_3_1/ > $OUT/pmc_3_1.txt; python3 scripts/pmc_summary.py $OUT/pmc_3_m1/ > $OUT/pmc_3_m1.txt; python3 scripts/pmc_summary.py $OUT/pmc_4_4/ > $OUT/pmc_4_4.txt
head -20 $OUT/pmc_3_1.txt $OUT/pmc_3_m1.txt $OUT/pmc_4_4.txt
