# Round-3 evidence of the build in the tree: full suite, smoke, bench, rocprof kernel trace, PMC (with the build tag),
# the other BASELINE configs and the frame-less profile, the two-rank rehearsal, and the diagnostics (segment
# shares, event counts). Each GPU step has its own time limit; a failing step ends the script.
R=$PWD; B=sphereflake-raytracer_amd; TAG=${1:-r3final}
bash scripts/round_profile.sh $TAG; rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
OUT=$R/gpurun_out/$TAG
bash scripts/configs_bench.sh $TAG/cfg > $OUT/configs.log 2>&1 || { tail -5 $OUT/configs.log; exit 7; }
grep -v "amdgpu\|^W20\|^E20" $OUT/configs.log | grep -E "^c[0-9]|batch"
bash scripts/multi_rehearsal.sh > $OUT/multi.log 2>&1 || { tail -5 $OUT/multi.log; exit 8; }
cp gpurun_out/multi/*.json $OUT/ 2>/dev/null
SF_LIB=$R/$B/build_phases/libsphereflake_hip.so timeout -k 10 120 python -u scripts/tile_schedule.py --reps 3 --out $OUT/tt_phases.npy > $OUT/phases.txt 2>&1 || exit 9
SF_LIB=$R/$B/build_counts/libsphereflake_hip.so timeout -k 10 120 python -u scripts/tile_schedule.py --reps 3 --counts --out $OUT/tt_counts.npy > $OUT/counts.txt 2>&1 || exit 10
grep -v amdgpu.ids $OUT/phases.txt $OUT/counts.txt
exit $rc
