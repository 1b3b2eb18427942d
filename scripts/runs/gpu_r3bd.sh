# The share-order test, then the full GPU suite.
R=$PWD; OUT=$R/gpurun_out/r3bd; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "member_share" --timeout 120 --timeout-method thread > $OUT/pytest_share.log 2>&1 || { tail -30 $OUT/pytest_share.log; exit 1; }
grep -E "PASSED|FAILED" $OUT/pytest_share.log | sed 's/.*:://' | tr '\n' ' '; echo
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 2; }
tail -1 $OUT/pytest_gpu.log
