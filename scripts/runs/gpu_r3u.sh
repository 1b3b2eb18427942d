# Frame-less: next batch's binning prefetched with its draws; draw segments probe.
R=$PWD; OUT=$R/gpurun_out/r3u; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash scripts/mt_seg_probe.sh r3u/mtseg || exit 5
exit $rc
