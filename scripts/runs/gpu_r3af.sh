R=$PWD; OUT=$R/gpurun_out/r3af; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/n8 -o run --output-format csv -- python3 $R/scripts/share_trace.py 8 3 300 > $OUT/n8.log 2>&1 || exit 1
grep "share-frame" $OUT/n8.log
head -8 $(find $OUT/n8 -name "*kernel_stats.csv") | cut -d, -f1-4,6,7
