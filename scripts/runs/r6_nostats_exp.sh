#!/bin/bash
# round 6 EXPERIMENT (measurement only, stats wrong): the per-wave stats publish skipped (SF_FLAGS=0x8000 on the
# build_exp library) -- how much of a 1/8 share's period is the waves' end-of-life latency?
set -o pipefail
O=gpurun_out/${TAG:-r6ns}; mkdir -p $O
EXP=$PWD/sphereflake-raytracer_amd/build_exp/libsphereflake_hip.so
for r in 1 2 3; do
  echo -n "main: " | tee -a $O/nostats.txt
  PROBE_N=1,8 timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | sed 's/.*\]: //' | tee -a $O/nostats.txt || exit 1
  echo -n "nostats: " | tee -a $O/nostats.txt
  SF_LIB_PARTIAL=1 SF_LIB=$EXP SF_FLAGS=0x8000 PROBE_N=1,8 timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | sed 's/.*\]: //' | tee -a $O/nostats.txt || exit 1
done
