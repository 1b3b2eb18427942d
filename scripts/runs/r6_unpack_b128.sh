#!/bin/bash
# round 6: the index-slab unpack with the child frames read as float4 columns (new) vs the library before
# (scratch_ab/lib_old.so): the slab tests, then the unpack alone, interleaved
set -o pipefail
O=gpurun_out/${TAG:-r6ub}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_group.py tests/test_gpu_random_views.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do
  for lib in old new; do
    if [ $lib = old ]; then export SF_LIB=$PWD/scratch_ab/lib_old.so; else unset SF_LIB; fi
    for W in "3840 2160 0.22" "1920 1080 0.25"; do
      timeout -k 10 200 python3 -u scripts/unpack_probe.py $W 8 50 2>&1 | grep unpack | sed "s/^/$lib /" | tee -a $O/unpack_ab.txt || exit 1
    done
  done
done
