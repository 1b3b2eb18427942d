# Self-test ties on a rare branch: parity, A/B vs HEAD; then scheduling knobs on the new kernel (slots,
# priority buckets).
R=$PWD; OUT=$R/gpurun_out/r3aa; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
REPS=4 PMC=1 scripts/lib_ab.sh r3aa/ab "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_prev/libsphereflake_hip.so || exit 5
for rep in 1 2; do
for k in "--slots 2" "--slots 4" "--slots 3"; do
  timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras $k > $OUT/k.json 2>/dev/null || exit 6
  python3 -c "import json; j=json.loads(open('$OUT/k.json').read().strip().split(chr(10))[-1]); print('$k', 'frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'lat', j['frame_latency_ms'])"
done
for pb in 0 4 12; do
  SF_PRIO_BUCKETS=$pb timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/k.json 2>/dev/null || exit 6
  python3 -c "import json; j=json.loads(open('$OUT/k.json').read().strip().split(chr(10))[-1]); print('prio $pb', 'frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'])"
done
done
exit $rc
