set -e
mkdir -p gpurun_out/spl1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "order or split" --timeout 120 --timeout-method thread > gpurun_out/spl1/pytest.log 2>&1 || { tail -30 gpurun_out/spl1/pytest.log; exit 1; }
tail -1 gpurun_out/spl1/pytest.log
scripts/ab_bench.sh spl1 "" "SF_SPLIT_BUCKETS=0" "SF_SPLIT_BUCKETS=1" "SF_SPLIT_BUCKETS=2" "SF_SPLIT_BUCKETS=3" "SF_SPLIT_PARTS=4 SF_SPLIT_BUCKETS=1" "SF_SPLIT_PARTS=4 SF_SPLIT_BUCKETS=2" "SF_SPLIT_PARTS=4 SF_SPLIT_BUCKETS=3"
