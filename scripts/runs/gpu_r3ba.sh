# Fixup workgroups without a tile return before the LDS setup: GPU tests, then shares / bench against the
# previous library (profiles' build, kept as build_prev/), interleaved.
R=$PWD; OUT=$R/gpurun_out/r3ba; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2; do
  for L in build_prev build; do
    SF_LIB=$R/sphereflake-raytracer_amd/$L/libsphereflake_hip.so PROBE_STEPS=1000 PROBE_N=1,4,8 PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/p.txt 2>&1 || exit 2
    echo "$L $(grep slots $OUT/p.txt)"
  done
done
