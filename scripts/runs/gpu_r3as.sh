# Is the bench's slower small share the torch-initialised runtime? share_probe with/without torch; share_bench
# with more hardware queues.
R=$PWD; OUT=$R/gpurun_out/r3as; mkdir -p $OUT
PROBE_N=4,8 PROBE_SLOTS=3,4 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/c.txt 2>&1 || exit 1
echo "share_probe"; grep -v amdgpu $OUT/c.txt
PROBE_TORCH=1 PROBE_N=4,8 PROBE_SLOTS=3,4 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/d.txt 2>&1 || exit 2
echo "share_probe with torch"; grep -v amdgpu $OUT/d.txt
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u scripts/share_bench.py 3,4 1,8 > $OUT/e.txt 2>&1 || exit 3
echo "share_bench, 8 HW queues"; grep -v amdgpu $OUT/e.txt
