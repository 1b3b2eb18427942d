#!/bin/bash
# Index-slab unpack with LDS-staged constants on resident workgroups: GPU suite, the unpack alone (4K / 1080p over
# 8), its PMC at 4K (two passes), the host cost of the slab-format decision.
set -e
R=$PWD; OUT=$R/gpurun_out/r5unpack; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
timeout -k 10 120 python3 -u scripts/unpack_probe.py 3840 2160 0.22 8 50 | grep unpack
timeout -k 10 120 python3 -u scripts/unpack_probe.py 1920 1080 0.25 8 50 | grep unpack
done > $OUT/unpack_alone.txt 2>&1; cat $OUT/unpack_alone.txt
timeout -k 10 120 python3 -u scripts/slab_bytes_probe.py 400 > $OUT/slab_bytes.txt 2>&1; grep views $OUT/slab_bytes.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVES -d $OUT/pmcu -o run --output-format csv -- python3 $R/scripts/unpack_probe.py 3840 2160 0.22 8 20 > $OUT/pmcu.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmcf -o run --output-format csv -- python3 $R/scripts/unpack_probe.py 3840 2160 0.22 8 20 > $OUT/pmcf.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmcw -o run --output-format csv -- python3 $R/scripts/unpack_probe.py 3840 2160 0.22 8 20 > $OUT/pmcw.log 2>&1
cd $R && python3 scripts/pmc_summary.py $OUT/pmcu $OUT/pmcf $OUT/pmcw > $OUT/pmc_unpack.txt 2>&1; grep -A12 "sf_slab_unpack4" $OUT/pmc_unpack.txt | head -14
