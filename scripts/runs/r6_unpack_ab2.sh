#!/bin/bash
# round 6: unpack tests, unpack probe A/B (round-6 base library vs the tree's), unpack PMC of the tree's library
set -o pipefail
O=gpurun_out/${TAG:-r6u2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_unpack.txt 2>&1 || { tail -30 $O/pytest_unpack.txt; exit 1; }
tail -1 $O/pytest_unpack.txt
BASE=$PWD/sphereflake-raytracer_amd/build_ab/lib_r6base.so
for r in 1 2; do
  for W in "3840 2160 0.22" "1920 1080 0.25"; do
    SF_LIB_PARTIAL=1 SF_LIB=$BASE timeout -k 10 200 python3 -u scripts/unpack_probe.py $W 8 50 2>&1 | grep unpack | sed 's/^/base /' | tee -a $O/unpack_ab.txt || exit 1
    timeout -k 10 200 python3 -u scripts/unpack_probe.py $W 8 50 2>&1 | grep unpack | sed 's/^/new  /' | tee -a $O/unpack_ab.txt || exit 1
  done
done
R=$PWD
cd /tmp && export TMPDIR=/tmp
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  n=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $R/$O/pmc_$n -o run --output-format csv -- python3 $R/scripts/unpack_probe.py 3840 2160 0.22 8 10 > $R/$O/pmc_$n.log 2>&1 || exit 1
done
python3 $R/scripts/pmc_summary.py $R/$O/pmc_*/ > $R/$O/pmc_unpack.txt 2>&1
grep -A18 "sf_slab_unpack4" $R/$O/pmc_unpack.txt | head -20
