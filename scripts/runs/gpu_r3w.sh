# Round evidence for the current build: full suite, smoke, bench, rocprof kernel trace, PMC (round_profile.sh),
# then the diagnostics of the same kernel (segment shares, event counts).
R=$PWD; B=sphereflake-raytracer_amd
bash scripts/round_profile.sh r3w; rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
OUT=$R/gpurun_out/r3w
SF_LIB=$R/$B/build_phases/libsphereflake_hip.so timeout -k 10 120 python -u scripts/tile_schedule.py --reps 3 --out $OUT/tt_phases.npy > $OUT/phases.txt 2>&1 || exit 7
SF_LIB=$R/$B/build_counts/libsphereflake_hip.so timeout -k 10 120 python -u scripts/tile_schedule.py --reps 3 --counts --out $OUT/tt_counts.npy > $OUT/counts.txt 2>&1 || exit 8
grep -v amdgpu.ids $OUT/phases.txt $OUT/counts.txt
exit $rc
