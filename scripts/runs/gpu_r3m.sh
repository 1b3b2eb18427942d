# diagnostics of the front-first build: segment shares (stamp build), event counts (count build), per-view times
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/r3m; mkdir -p $OUT
B=sphereflake-raytracer_amd
SF_LIB=$R/$B/build_phases/libsphereflake_hip.so timeout -k 10 120 python -u scripts/tile_schedule.py --reps 3 --out $OUT/tt_phases.npy > $OUT/phases.txt 2>&1 || exit 3
grep -v amdgpu.ids $OUT/phases.txt
SF_LIB=$R/$B/build_counts/libsphereflake_hip.so timeout -k 10 120 python -u scripts/tile_schedule.py --reps 3 --counts --out $OUT/tt_counts.npy > $OUT/counts.txt 2>&1 || exit 4
grep -v amdgpu.ids $OUT/counts.txt
SF_LIB=$R/$B/build_counts/libsphereflake_hip.so SF_FLAGS=0x100 timeout -k 10 120 python -u scripts/tile_schedule.py --reps 3 --counts --out $OUT/tt_counts0.npy > $OUT/counts_nocull.txt 2>&1 || exit 4
grep -v amdgpu.ids $OUT/counts_nocull.txt
timeout -k 10 200 python -u scripts/view_probe.py 3 > $OUT/views.txt 2>&1 || exit 5
grep -v amdgpu.ids $OUT/views.txt
