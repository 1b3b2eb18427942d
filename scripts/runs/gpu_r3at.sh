# Fused order scan + scatter for small orders: GPU tests, then the share probes (with / without torch, share_bench).
R=$PWD; OUT=$R/gpurun_out/r3at; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
bash scripts/gpu_r3as.sh
