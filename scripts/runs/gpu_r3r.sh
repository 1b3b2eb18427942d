# fast LOD decisions in the child tests: parity suite, then A/B against HEAD (build_base)
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/r3r; mkdir -p $OUT
B=sphereflake-raytracer_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=4 PMC=1 scripts/lib_ab.sh r3r/ab "" $B/build/libsphereflake_hip.so $B/build_base/libsphereflake_hip.so || exit 5
exit $rc
