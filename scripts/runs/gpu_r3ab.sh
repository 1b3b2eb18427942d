# Per-tile arithmetic: u = x / W by reciprocal + fma correction, tile divmod by magic numbers: parity, A/B
R=$PWD; OUT=$R/gpurun_out/r3ab; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
REPS=4 PMC=1 scripts/lib_ab.sh r3ab/ab "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_prev/libsphereflake_hip.so || exit 5
exit $rc
