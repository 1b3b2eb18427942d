# Kernel trace of a member's 1/8 share at 1 and 3 frames in flight (where the small share's frame time goes).
R=$PWD; OUT=$R/gpurun_out/r3am; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for s in 1 3; do
  timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT/s$s -o run --output-format csv -- python3 $R/scripts/share_trace.py 8 $s 300 > $OUT/s$s.log 2>&1 || exit 1
  f=$(ls $OUT/s$s/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/s$s/run_kernel_trace.csv)
  echo "== slots $s"; grep "share-frame" $OUT/s$s.log; python3 $R/scripts/trace_overlap.py $f 350
done
