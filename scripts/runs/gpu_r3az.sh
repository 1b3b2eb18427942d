# What the fixup launch costs a frame (experiment library exp_nofix/: SF_EXP_NO_FIXUP=1 skips it on bounded
# renders; ties unhandled, measurement only): shares and the whole frame, interleaved.
R=$PWD; OUT=$R/gpurun_out/r3az; mkdir -p $OUT
L=$R/exp_nofix/build/libsphereflake_hip.so
for rep in 1 2; do
  for v in "SF_NONE=0" "SF_EXP_NO_FIXUP=1"; do
    env $v SF_LIB=$L PROBE_STEPS=1000 PROBE_N=1,4,8 PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/p.txt 2>&1 || exit 1
    echo "$v $(grep slots $OUT/p.txt)"
    env $v SF_LIB=$L timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/b.json 2>/dev/null || exit 2
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$v bench frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'lat', j['frame_latency_ms'])"
  done
done
