set -e
mkdir -p gpurun_out/diag
timeout -k 10 120 python scripts/tile_schedule.py --out gpurun_out/diag/tt_w4.npy > gpurun_out/diag/tt_w4.txt 2>&1
SF_TRACE_WAVES=1 timeout -k 10 120 python scripts/tile_schedule.py --out gpurun_out/diag/tt_w1.npy > gpurun_out/diag/tt_w1.txt 2>&1
SF_TRACE_WAVES=1 SF_LIB=$PWD/sphereflake-raytracer_amd/build_phases/libsphereflake_hip.so timeout -k 10 120 python scripts/tile_schedule.py --out gpurun_out/diag/tt_ph.npy > gpurun_out/diag/tt_ph.txt 2>&1
cat gpurun_out/diag/*.txt
