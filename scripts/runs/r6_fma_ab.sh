#!/bin/bash
# round 6: GPU suite on the exact-fma / unpack build, bench A/B against the round-6 base library, unpack PMC passes
set -o pipefail
O=gpurun_out/r6f1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
REPS=3 scripts/lib_ab.sh r6f1/ab "" sphereflake-raytracer_amd/build_ab/lib_r6base.so sphereflake-raytracer_amd/build/libsphereflake_hip.so 2>&1 | tee $O/ab.txt || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
for L in base new; do
  LIB=$R/sphereflake-raytracer_amd/build/libsphereflake_hip.so; [ $L = base ] && LIB=$R/sphereflake-raytracer_amd/build_ab/lib_r6base.so
  for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    n=$(echo $P | cut -d' ' -f1)
    SF_LIB_PARTIAL=1 SF_LIB=$LIB timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $R/$O/pmc_${L}_$n -o run --output-format csv -- python3 $R/scripts/unpack_probe.py 3840 2160 0.22 8 10 > $R/$O/pmc_${L}_$n.log 2>&1 || exit 1
  done
  python3 $R/scripts/pmc_summary.py $R/$O/pmc_${L}_*/ > $R/$O/pmc_unpack_$L.txt 2>&1
  grep -A20 "sf_slab_unpack4" $R/$O/pmc_unpack_$L.txt | head -24
done
