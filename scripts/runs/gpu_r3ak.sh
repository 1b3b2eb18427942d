# Host enqueue cost per frame against the share's frame period (is a small share host-bound?).
R=$PWD; OUT=$R/gpurun_out/r3ak; mkdir -p $OUT
PROBE_SLOTS=1,3 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/share.txt 2>&1 || exit 1
grep -v amdgpu $OUT/share.txt
PROBE_SLOTS=1,3 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py 64 64 0.25 > $OUT/tiny.txt 2>&1 || exit 2
grep -v amdgpu $OUT/tiny.txt
