# front-first order: parity suite, then default vs index order (0x200) vs no cull (0x100), timing + PMC
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/r3l; mkdir -p $OUT
L=sphereflake-raytracer_amd/build/libsphereflake_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=3 PMC=1 scripts/lib_ab.sh r3l/occl "" $L@0 $L@0x200 $L@0x100 || exit 5
exit $rc
