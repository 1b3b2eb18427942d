# Diagnostics: traversal event counts (COUNTS=1 build) at the bench config
set -e
mkdir -p gpurun_out/cnt
SF_LIB=$PWD/sphereflake-raytracer_amd/build_counts/libsphereflake_hip.so timeout -k 10 120 python scripts/tile_schedule.py --reps 2 --counts --out gpurun_out/cnt/t.npy > gpurun_out/cnt/counts.txt 2>&1
grep -v amdgpu.ids gpurun_out/cnt/counts.txt
