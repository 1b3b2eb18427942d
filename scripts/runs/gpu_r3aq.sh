# A member's share through bench.py's own timed loop (scripts/share_bench.py): slots 3/4/5, N = 1, 4, 8.
R=$PWD; OUT=$R/gpurun_out/r3aq; mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/share_bench.py 3,4,5 1,4,8 > $OUT/sb.txt 2>&1; rc=$?
grep -v amdgpu $OUT/sb.txt; exit $rc
