#!/bin/bash
# Round 4: the cone cull skipped for nodes small against the cone (SF_CONE_SKIP = k): parity with k = 16 on the
# tree, then interleaved timing of lane32.so (no test) and the tree at k = 0 / 4 / 16 / 64, PMC at 0 and 16.
R=$PWD; OUT=$R/gpurun_out/r4y; mkdir -p $OUT
SF_CONE_SKIP=16 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 5; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2 3; do
  for v in "lane32 build_ab/lane32.so 0" "k0 build_ab/coneskip.so 0" "k4 build_ab/coneskip.so 4" "k16 build_ab/coneskip.so 16" "k64 build_ab/coneskip.so 64"; do
    set -- $v
    SF_CONE_SKIP=$3 SF_LIB_PARTIAL=1 SF_LIB=$R/sphereflake-raytracer_amd/$2 timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 7; }
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$1', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'clk', j['roofline'].get('clock_mhz_live'), 'fixed', j['fixed_camera']['frame_ms'], 'check', j['check']['bit_exact'])"
  done
done
for k in 0 16; do
  for cfg in "c4 3840 2160 0.22" "c5 16384 16384 0.2"; do
    set -- $cfg
    EXTRA=""; [ $1 = c5 ] && EXTRA="--steps 10 --warmup 3"
    SF_CONE_SKIP=$k timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-extras --width $2 --height $3 --K $4 $EXTRA > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 8; }
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$1 k$k', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'clk', j['roofline'].get('clock_mhz_live'), 'check', j['check']['bit_exact'])"
  done
done
cd /tmp && export TMPDIR=/tmp
for k in 0 16; do
  SF_CONE_SKIP=$k timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES -d $OUT/pmc$k -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > $OUT/pmc$k.log 2>&1
  echo "== k=$k"; python3 $R/scripts/pmc_summary.py $OUT/pmc$k | grep -A6 "sf_trace_queue2 " || true
done
