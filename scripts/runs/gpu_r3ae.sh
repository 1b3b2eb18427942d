# A member's share at more frames in flight with more hardware queues (GPU_MAX_HW_QUEUES).
R=$PWD; OUT=$R/gpurun_out/r3ae; mkdir -p $OUT
PROBE_SLOTS=3,4,6,8 PROBE_SPLITS=auto,model timeout -k 10 600 python3 -u scripts/share_probe.py > $OUT/share_1080.txt 2>&1 || { tail -5 $OUT/share_1080.txt; exit 1; }
grep -v amdgpu $OUT/share_1080.txt
PROBE_SLOTS=3,6 PROBE_SPLITS=auto timeout -k 10 600 python3 -u scripts/share_probe.py 3840 2160 0.22 > $OUT/share_4k.txt 2>&1 || exit 2
grep -v amdgpu $OUT/share_4k.txt
