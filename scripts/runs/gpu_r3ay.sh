# Does the bench loop's kernel timing (events + clock probe every k-th render) cost throughput? share_bench with
# and without it, slots 3 and 4, N = 1 and 8.
R=$PWD; OUT=$R/gpurun_out/r3ay; mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/share_bench.py 3,4 1,8 > $OUT/a.txt 2>&1 || exit 1
echo "timing on"; grep -v amdgpu $OUT/a.txt
SHARE_NO_TIMING=1 timeout -k 10 300 python3 -u scripts/share_bench.py 3,4 1,8 > $OUT/b.txt 2>&1 || exit 2
echo "timing off"; grep -v amdgpu $OUT/b.txt
