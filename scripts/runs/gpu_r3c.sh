set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r3c/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r3c/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/r3c/bench_quick.json 2> gpurun_out/r3c/bench_quick.err || { tail -30 gpurun_out/r3c/bench_quick.err; exit 4; }
tail -1 gpurun_out/r3c/bench_quick.json
PMC=1 scripts/lib_ab.sh r3c_lds "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_x1/libsphereflake_hip.so
timeout -k 10 300 python -u scripts/share_probe.py > gpurun_out/r3c/share_1080.txt 2>&1 || exit 6
cat gpurun_out/r3c/share_1080.txt
timeout -k 10 300 python -u scripts/share_probe.py 3840 2160 0.22 > gpurun_out/r3c/share_4k.txt 2>&1 || exit 6
cat gpurun_out/r3c/share_4k.txt
