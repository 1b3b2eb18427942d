# Order only on frames of at most half the grid's waves: GPU tests, bench (default), configs, shares.
R=$PWD; OUT=$R/gpurun_out/r3ax; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/b.json 2>/dev/null || exit 4
  python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('default 1080p frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'lat', j['frame_latency_ms'], 'Mrays', j['value'])"
done
for cfg in "c1 640 360 1.0" "c2 1280 720 0.8"; do
  set -- $cfg
  timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --width $2 --height $3 --K $4 > $OUT/b.json 2> $OUT/b.err || exit 5
  python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$1', 'frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'lat', j['frame_latency_ms'])"
done
PROBE_STEPS=1000 PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/p.txt 2>&1 || exit 6
grep -v amdgpu $OUT/p.txt
