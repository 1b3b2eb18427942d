#!/bin/bash
# Parity gate on the GPU box for the library as built in-tree: the full -m gpu suite, smoke(), and the
# default bench line, each under its own time limit; stops at the first failure.
# Usage (on the box, from the repo root): scripts/head_check.sh <tag>
set -e
TAG=${1:-head}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cp -f BUILD_SHA $OUT/ 2>/dev/null || true
sha256sum sphereflake-raytracer_amd/build/libsphereflake_hip.so > $OUT/lib_sha256.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json
