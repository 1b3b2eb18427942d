# In-kernel tie re-trace (fixup_inline): the tie-fallback tests first (forced re-trace, both paths), the full GPU
# suite, then shares and the whole frame against the previous library (build_prev/), interleaved.
R=$PWD; OUT=$R/gpurun_out/r3bb; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "tie_fallback" --timeout 120 --timeout-method thread > $OUT/pytest_tie.log 2>&1 || { tail -30 $OUT/pytest_tie.log; exit 1; }
grep -E "PASSED|FAILED" $OUT/pytest_tie.log | sed 's/.*:://' | tr '\n' ' '; echo
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2; do
  for L in build_prev build; do
    SF_LIB=$R/sphereflake-raytracer_amd/$L/libsphereflake_hip.so PROBE_STEPS=1000 PROBE_N=1,2,4,8 PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/p.txt 2>&1 || exit 3
    echo "$L $(grep slots $OUT/p.txt)"
  done
done
for L in build_prev build; do
  SF_LIB_PARTIAL=1 SF_LIB=$R/sphereflake-raytracer_amd/$L/libsphereflake_hip.so timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/b.json 2>/dev/null || exit 4
  python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$L bench frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'lat', j['frame_latency_ms'])"
done
