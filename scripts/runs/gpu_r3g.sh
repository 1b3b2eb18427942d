# parity suite on the skewed table / lane-31 centre layout, then the LDS A/B (timing + PMC) against build_base
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/r3g; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
REPS=3 PMC=1 scripts/lib_ab.sh r3g/lds "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_base/libsphereflake_hip.so
