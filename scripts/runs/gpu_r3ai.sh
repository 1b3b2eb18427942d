# Defaults: tile order only for frames that fill the grid at most twice, 4 tile queues per XCD: parity, bench
# (default config), the other configs, a member's share (1..8 GPUs).
R=$PWD; OUT=$R/gpurun_out/r3ai; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/b.json 2>/dev/null || exit 4
  python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('default 1080p frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'lat', j['frame_latency_ms'], 'Mrays', j['value'])"
done
bash scripts/configs_bench.sh r3ai/cfg 2>&1 | grep -E "^c[0-9]|batch  262144"
PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 600 python3 -u scripts/share_probe.py > $OUT/share_1080.txt 2>&1 || exit 6
grep -v amdgpu $OUT/share_1080.txt
exit $rc
