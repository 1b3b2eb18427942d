#!/bin/bash
# Round-6 multi-frame trace: the loop-shape probe at 1080p and for a 1/8 share, per-frame launches against batches,
# for several interleaved-head sizes (SF_FRAMES_HEAVY).
set -o pipefail
OUT=$PWD/gpurun_out/${1:-r6f}
mkdir -p $OUT
export TMPDIR=/tmp
for h in 0 64 256 1024; do
  SF_FRAMES_HEAVY=$h timeout -k 10 200 python -u scripts/frames_probe.py 1920 1080 0.25 --configs "3:1,8:4,16:8" > $OUT/probe_1080_h$h.txt 2>&1
  rc=$?; echo "heavy $h"; grep share $OUT/probe_1080_h$h.txt; [ $rc -ne 0 ] && exit $rc
done
for h in 0 64 256; do
  SF_FRAMES_HEAVY=$h timeout -k 10 200 python -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --configs "4:1,8:8,16:8" > $OUT/probe_share8_h$h.txt 2>&1
  rc=$?; echo "heavy $h"; grep share $OUT/probe_share8_h$h.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
