# Occlusion radius without the square root (per-lane bound from tca), cull_t hoisted: parity, A/B vs HEAD.
R=$PWD; OUT=$R/gpurun_out/r3y; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
REPS=4 PMC=1 scripts/lib_ab.sh r3y/ab "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_osq/libsphereflake_hip.so sphereflake-raytracer_amd/build_prev/libsphereflake_hip.so || exit 5
exit $rc
