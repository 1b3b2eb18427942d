#!/bin/bash
# Round 5: the slot-residency rehearsal, the 4K rows-mode unpack under a kernel trace, the 4K share probe.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5i
mkdir -p $OUT
timeout -k 10 180 python3 -u scripts/slot_residency_probe.py 20 > $OUT/slot_residency.txt 2>&1
cat $OUT/slot_residency.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rows4k -o run --output-format csv -- python3 $R/bench.py --mode rows --gpus 8 --width 3840 --height 2160 --K 0.22 --steps 30 --warmup 5 --no-cpu-baseline --no-extras > $OUT/rows4k.json 2> $OUT/rows4k.err
python3 $R/scripts/unpack_overlap.py $(find $OUT/rows4k -name "*kernel_trace.csv") | tee $OUT/rows4k_overlap.txt
grep -E "sf_slab_unpack|sf_trace|sf_node" $(find $OUT/rows4k -name "*kernel_stats.csv") | tee $OUT/rows4k_stats.txt
cd $R
timeout -k 10 400 python3 -u scripts/share_probe.py 3840 2160 0.22 > $OUT/share4k.txt 2>&1
cat $OUT/share4k.txt
