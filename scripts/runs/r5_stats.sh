#!/bin/bash
# Stats written by the trace's last wave (no copy after the trace): GPU suite, lone-frame timeline, bench lines;
# PMC of the 4K index-slab unpack alone.
set -e
R=$PWD; OUT=$R/gpurun_out/r5stats; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python3 -u scripts/lone_frame_timeline.py > $OUT/plain.txt 2>&1; grep lone $OUT/plain.txt
for st in 20 200; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps $st --warmup 5 > $OUT/b_$st.json 2>/dev/null
  python3 -c "import json; j=json.loads(open('$OUT/b_$st.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print($st, 'frame', j['frame_ms'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', j['frame_latency_ms'], 'exact', j['check']['bit_exact'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/tr -o run -- python3 $R/scripts/lone_frame_timeline.py > $OUT/traced.txt 2>&1
cd $R && python3 scripts/lone_frame_timeline.py --report $OUT/tr > $OUT/report.txt 2>&1; head -9 $OUT/report.txt; rm -rf $OUT/tr
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVES -d $OUT/pmcu -o run --output-format csv -- python3 $R/scripts/unpack_probe.py 3840 2160 0.22 8 20 > $OUT/pmcu.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE WRITE_SIZE -d $OUT/pmcu2 -o run --output-format csv -- python3 $R/scripts/unpack_probe.py 3840 2160 0.22 8 20 > $OUT/pmcu2.log 2>&1
cd $R && python3 scripts/pmc_summary.py $OUT/pmcu $OUT/pmcu2 > $OUT/pmc_unpack.txt 2>&1; grep -A12 "sf_slab_unpack4" $OUT/pmc_unpack.txt | head -30
