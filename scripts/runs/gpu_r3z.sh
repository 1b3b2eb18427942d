# Child loop scalar bookkeeping (entry order as bit order, direct continue on no bounding hit; + depth offset
# and table offset carried): parity, A/B vs HEAD.
R=$PWD; OUT=$R/gpurun_out/r3z; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
REPS=4 PMC=1 scripts/lib_ab.sh r3z/ab "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_c1/libsphereflake_hip.so sphereflake-raytracer_amd/build_prev/libsphereflake_hip.so || exit 5
exit $rc
