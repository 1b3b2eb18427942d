set -e
mkdir -p gpurun_out/v14
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v14/smoke.log 2>&1 || { tail -5 gpurun_out/v14/smoke.log; exit 1; }
tail -1 gpurun_out/v14/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v14/pytest.log 2>&1 || { tail -30 gpurun_out/v14/pytest.log; exit 1; }
tail -2 gpurun_out/v14/pytest.log
scripts/sweep.sh v14sw "SF_ORDER=0" "SF_ORDER=1" "SF_ORDER=1 SF_TRACE_WAVES=1" "SF_ORDER=1 SF_TRACE_WAVES=4"
