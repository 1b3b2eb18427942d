# Host cost per frame by launches per render (order kernels off: SF_ORDER=0; fixup off: SF_FLAGS=0x200, which
# drops the front-first order so a bounded render launches no fixup), then the 1/8 share at more frames in flight.
R=$PWD; OUT=$R/gpurun_out/r3an; mkdir -p $OUT
for v in "SF_NONE=0" "SF_ORDER=0" "SF_ORDER=0 SF_FLAGS=0x200"; do
  echo "== $v"; env $v timeout -k 10 300 python3 -u scripts/host_cost_probe.py > $OUT/host.txt 2>&1 || exit 1
  grep -v amdgpu $OUT/host.txt
done
PROBE_SLOTS=3,4,6 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/share.txt 2>&1 || exit 2
grep -v amdgpu $OUT/share.txt
SF_SPLIT_BUCKETS=0 PROBE_SLOTS=4,6 PROBE_SPLITS=0 timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/share0.txt 2>&1 || exit 3
grep -v amdgpu $OUT/share0.txt
