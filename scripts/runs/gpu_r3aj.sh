# A member's share of the frame at more frames in flight with more hardware queues per process, and without the
# order on the share (SF_ORDER=0).
R=$PWD; OUT=$R/gpurun_out/r3aj; mkdir -p $OUT
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q PROBE_SLOTS=3,6,8 PROBE_SPLITS=auto timeout -k 10 600 python3 -u scripts/share_probe.py > $OUT/share_q$q.txt 2>&1 || exit 1
  echo "== GPU_MAX_HW_QUEUES=$q"; grep -v amdgpu $OUT/share_q$q.txt
done
SF_ORDER=0 PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 600 python3 -u scripts/share_probe.py > $OUT/share_noorder.txt 2>&1 || exit 2
echo "== SF_ORDER=0"; grep -v amdgpu $OUT/share_noorder.txt
