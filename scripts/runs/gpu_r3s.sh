# Round-3 session 2: parity of the tighter occlusion margin (3 x 2^-10) and the communicator-less multi-rank
# bands, bench line, interleaved A/B against the 2^-7 margin build, the two-rank bench rehearsal.
R=$PWD; OUT=$R/gpurun_out/r3s; mkdir -p $OUT
git_sha=$(cat BUILD_SHA 2>/dev/null); echo "tree $git_sha" > $OUT/build_info.txt
python3 -c "import sys; sys.path.insert(0, 'sphereflake-raytracer_amd'); import sphereflake_amd as sf; print(sf.build_info())" >> $OUT/build_info.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
tail -1 $OUT/bench.json
REPS=4 PMC=1 scripts/lib_ab.sh r3s/ab "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_base/libsphereflake_hip.so sphereflake-raytracer_amd/build_fsq/libsphereflake_hip.so || exit 5
bash scripts/multi_rehearsal.sh > $OUT/multi.log 2>&1; m=$?
tail -5 $OUT/multi.log
exit $(( rc > 0 ? rc : m ))
