# Knobs on a member's share at 4 frames in flight (1/4 and 1/8 of 1080p).
R=$PWD; OUT=$R/gpurun_out/r3ao; mkdir -p $OUT
for v in "SF_NONE=0" "SF_PIPE=0" "SF_ORDER=0" "SF_ORDER=0 SF_PIPE=0" "SF_ORDER_EVERY=6" "SF_PRIO_BUCKETS=0" "SF_NONE=0"; do
  env $v PROBE_N=1,4,8 PROBE_SLOTS=4 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/p.txt 2>&1 || exit 1
  echo "$v $(grep slots $OUT/p.txt)"
done
