# share_bench with and without the trace-kernel timing events, slots 3, N = 4, 8.
R=$PWD; OUT=$R/gpurun_out/r3ar; mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/share_bench.py 3 4,8 > $OUT/a.txt 2>&1 || exit 1
echo "timing on"; grep -v amdgpu $OUT/a.txt
SHARE_NO_TIMING=1 timeout -k 10 300 python3 -u scripts/share_bench.py 3 4,8 > $OUT/b.txt 2>&1 || exit 2
echo "timing off"; grep -v amdgpu $OUT/b.txt
PROBE_N=4,8 PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/c.txt 2>&1 || exit 3
echo "share_probe"; grep -v amdgpu $OUT/c.txt
