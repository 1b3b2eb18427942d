# Member shares row-major by default: GPU suite, shares N = 1..8 (interleaved with SF_ORDER=1), bench.
R=$PWD; OUT=$R/gpurun_out/r3bc; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2; do
  for v in "SF_NONE=0" "SF_ORDER=1"; do
    env $v PROBE_STEPS=1000 PROBE_N=1,2,4,8 PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/p.txt 2>&1 || exit 2
    echo "$v $(grep slots $OUT/p.txt)"
  done
done
