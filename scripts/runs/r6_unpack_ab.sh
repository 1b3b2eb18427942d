set -o pipefail
O=gpurun_out/r6u1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_unpack.txt 2>&1 || { tail -30 $O/pytest_unpack.txt; exit 1; }
tail -2 $O/pytest_unpack.txt
for r in 1 2; do
  SF_LIB_PARTIAL=1 SF_LIB=$PWD/sphereflake-raytracer_amd/build_ab/lib_r6base.so timeout -k 10 200 python3 -u scripts/unpack_probe.py 3840 2160 0.22 8 50 2>&1 | sed 's/^/base /' | tee -a $O/unpack_ab.txt || exit 1
  timeout -k 10 200 python3 -u scripts/unpack_probe.py 3840 2160 0.22 8 50 2>&1 | sed 's/^/new  /' | tee -a $O/unpack_ab.txt || exit 1
  SF_LIB_PARTIAL=1 SF_LIB=$PWD/sphereflake-raytracer_amd/build_ab/lib_r6base.so timeout -k 10 200 python3 -u scripts/unpack_probe.py 1920 1080 0.25 8 50 2>&1 | sed 's/^/base /' | tee -a $O/unpack_ab.txt || exit 1
  timeout -k 10 200 python3 -u scripts/unpack_probe.py 1920 1080 0.25 8 50 2>&1 | sed 's/^/new  /' | tee -a $O/unpack_ab.txt || exit 1
done
