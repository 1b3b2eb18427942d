# event counts of the front-first build (wholly culled entries), then product vs child-loop cull experiment
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/r3n; mkdir -p $OUT
B=sphereflake-raytracer_amd
SF_LIB=$R/$B/build_counts/libsphereflake_hip.so timeout -k 10 120 python -u scripts/tile_schedule.py --reps 3 --counts --out $OUT/tt.npy > $OUT/counts.txt 2>&1 || exit 3
grep -v amdgpu.ids $OUT/counts.txt
REPS=3 PMC=1 scripts/lib_ab.sh r3n/ab "" $B/build/libsphereflake_hip.so $B/build_exp/libsphereflake_hip.so
