#!/bin/bash
# Round 4: the order tests under the new rule, the BASELINE configs, the lone-frame latency probe.
R=$PWD; OUT=$R/gpurun_out/r4e; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "order or split or tie" --timeout 120 --timeout-method thread > $OUT/pytest_order.log 2>&1
rc=$?; tail -2 $OUT/pytest_order.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
grep -E "^FAILED|^ERROR" $OUT/pytest_order.log | head -20
SF_FLAGS=0x20 timeout -k 10 120 python3 -u scripts/latency_probe.py > $OUT/latency.txt 2>&1 || { tail -5 $OUT/latency.txt; exit 3; }
grep frame $OUT/latency.txt
bash scripts/configs_bench.sh r4e/cfg > $OUT/configs.log 2>&1 || { tail -5 $OUT/configs.log; exit 7; }
grep -E "^c[0-9]|batch" $OUT/configs.log
exit $rc
