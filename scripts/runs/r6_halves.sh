#!/bin/bash
# round 6: row-major half-tile units (SF_HALVES=1) -- parity with the env set, then the 1080p shares A/B
set -o pipefail
O=gpurun_out/${TAG:-r6h}; mkdir -p $O
SF_HALVES=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_views.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_halves.txt 2>&1 || { tail -30 $O/pytest_halves.txt; exit 1; }
tail -1 $O/pytest_halves.txt
for r in 1 2; do
  PROBE_N=1,4,8 timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | sed 's/^/base   /' | tee -a $O/share.txt || exit 1
  SF_HALVES=1 PROBE_N=1,4,8 timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | sed 's/^/halves /' | tee -a $O/share.txt || exit 1
done
