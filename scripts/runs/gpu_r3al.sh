# Host cost per call of SetView / Render / dist frames (scripts/host_cost_probe.py).
R=$PWD; OUT=$R/gpurun_out/r3al; mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/host_cost_probe.py > $OUT/host.txt 2>&1; rc=$?
grep -v amdgpu $OUT/host.txt; exit $rc
