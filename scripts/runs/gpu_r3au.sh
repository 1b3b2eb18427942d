# Why the bench loop's small share is slower than share_probe's: settle time and run length.
R=$PWD; OUT=$R/gpurun_out/r3au; mkdir -p $OUT
SHARE_SETTLE_MS=0 timeout -k 10 300 python3 -u scripts/share_bench.py 3,4 1,8 > $OUT/a.txt 2>&1 || exit 1
echo "share_bench settle 0"; grep -v amdgpu $OUT/a.txt
PROBE_STEPS=200 PROBE_WARM=6000 PROBE_N=8 PROBE_SLOTS=3,4 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/b.txt 2>&1 || exit 2
echo "share_probe warm 6000"; grep -v amdgpu $OUT/b.txt
PROBE_STEPS=2000 PROBE_WARM=30 PROBE_N=8 PROBE_SLOTS=3,4 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/c.txt 2>&1 || exit 3
echo "share_probe steps 2000"; grep -v amdgpu $OUT/c.txt
