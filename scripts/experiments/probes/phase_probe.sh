# Diagnostics: DFS segment shares (stamp build), uncontended (1 wave/CU) and full occupancy
set -e
mkdir -p gpurun_out/ph
for B in 128 0; do
  SF_MAX_BLOCKS=$B SF_LIB=$PWD/sphereflake-raytracer_amd/build_phases/libsphereflake_hip.so timeout -k 10 120 python scripts/tile_schedule.py --reps 2 --out gpurun_out/ph/b$B.npy > gpurun_out/ph/b$B.txt 2>&1
  echo "blocks=$B"; cat gpurun_out/ph/b$B.txt | grep -v amdgpu.ids
done
