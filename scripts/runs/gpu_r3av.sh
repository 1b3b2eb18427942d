# sf_dist vs plain contexts for a member's share, same loop (scripts/share_loop_probe.py).
R=$PWD; OUT=$R/gpurun_out/r3av; mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/share_loop_probe.py 8 3,4 2000 > $OUT/a.txt 2>&1; rc=$?
grep -v amdgpu $OUT/a.txt; exit $rc
