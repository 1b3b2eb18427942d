#!/bin/bash
# Parity gate on the GPU box for the library as built in-tree: the full -m gpu suite, smoke(), the default
# bench line, then optional probes, each under its own time limit. A test FAILURE (pytest exit 1) still lets
# the bench run; a time limit, crash or signal ends the script there.
# Usage (on the box, from the repo root): scripts/head_check.sh <tag> [probe ...]
#   probes: overlap (scripts/overlap_probe.py at 1080p and 4K)
TAG=${1:-head}; shift || true
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cp -f BUILD_SHA $OUT/ 2>/dev/null || true
sha256sum sphereflake-raytracer_amd/build/libsphereflake_hip.so > $OUT/lib_sha256.txt
python3 -c "import sys; sys.path.insert(0, 'sphereflake-raytracer_amd'); import sphereflake_amd as sf; print(sf.build_info())" > $OUT/build_info.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
cat $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 4; }
tail -1 $OUT/bench.json
for p in "$@"; do
  case $p in
    overlap)
      timeout -k 10 200 python -u scripts/overlap_probe.py > $OUT/overlap_1080.txt 2>&1 || exit 5
      cat $OUT/overlap_1080.txt
      timeout -k 10 200 python -u scripts/overlap_probe.py 3840 2160 0.22 > $OUT/overlap_4k.txt 2>&1 || exit 5
      cat $OUT/overlap_4k.txt ;;
  esac
done
exit $rc
