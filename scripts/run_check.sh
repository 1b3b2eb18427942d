set -e
T=${1:-v28}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "forking or heavy_first" > gpurun_out/$T/pytest_fork.log 2>&1 || { tail -30 gpurun_out/$T/pytest_fork.log; exit 1; }
tail -2 gpurun_out/$T/pytest_fork.log
bash scripts/count_probe.sh
scripts/sweep.sh ${T}sw "SF_FORK=0" "SF_FORK=1" "SF_FLAGS=8" "SF_FORK_DEPTH=2" "SF_FORK_DEPTH=4" "SF_FORK_TILES=64" "SF_FORK_TILES=1024"
