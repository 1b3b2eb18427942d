# Parity of the squared-form cone cull + fast sqrt_rn self test (product build), interleaved A/B against the
# margin-only and margin+fast-sqrt builds, then the other BASELINE configs and the frame-less profile.
R=$PWD; OUT=$R/gpurun_out/r3t; mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'sphereflake-raytracer_amd'); import sphereflake_amd as sf; print(sf.build_info())" > $OUT/build_info.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
REPS=4 PMC=1 scripts/lib_ab.sh r3t/ab "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_m/libsphereflake_hip.so sphereflake-raytracer_amd/build_fsq/libsphereflake_hip.so || exit 5
bash scripts/configs_bench.sh r3t/cfg || exit 6
exit $rc
