# Immediate-entry per-ray traversal: full parity suite, interleaved A/B against the test-all-then-enter build,
# configs c1/c2 (the latency variant shares the new loop now).
R=$PWD; OUT=$R/gpurun_out/r3x; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
if [ $rc -ne 0 ]; then exit $rc; fi
REPS=4 PMC=1 scripts/lib_ab.sh r3x/ab "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_old/libsphereflake_hip.so || exit 5
for L in build build_old; do for cfg in "c1 640 360 1.0" "c2 1280 720 0.8"; do set -- $cfg
  SF_LIB=$R/sphereflake-raytracer_amd/$L/libsphereflake_hip.so timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --width $2 --height $3 --K $4 > $OUT/b_$L_$1.json 2>/dev/null || exit 6
  python3 -c "import json; j=json.loads(open('$OUT/b_$L_$1.json').read().strip().split(chr(10))[-1]); print('$L $1', 'frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'])"
done; done
exit $rc
