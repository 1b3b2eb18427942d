# Frame-less batch time against the number of jump-ahead draw segments (SF_MT_SEGMENTS), prefetch on:
# fewer segments = less chip work competing with the trace, longer (hidden) draw latency.
R=$PWD; OUT=$R/gpurun_out/${1:-mtseg}; mkdir -p $OUT
for k in 32 16 8 4 2; do
  echo "== SF_MT_SEGMENTS=$k"
  SF_MT_SEGMENTS=$k timeout -k 10 120 python3 -u scripts/prog_bench.py 2>&1 | grep -v amdgpu | grep 262144 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for k in 32 4; do
  SF_MT_SEGMENTS=$k timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$k -o run --output-format csv -- python3 $R/scripts/prog_bench.py > $OUT/prof_$k.log 2>&1 || exit 2
  echo "== rocprof SF_MT_SEGMENTS=$k"; head -12 $(find $OUT/prof_$k -name "*kernel_stats.csv") | cut -d, -f1-4
done
