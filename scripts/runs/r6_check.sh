#!/bin/bash
# Round-6 GPU check: the full -m gpu suite, then smoke, on the tree as it is (library prebuilt in-tree).
# Usage (from the repo root, via gpurun): bash scripts/r6_check.sh <tag>
set -o pipefail
TAG=${1:-r6}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
tail -2 $OUT/smoke.txt
