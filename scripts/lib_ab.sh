#!/bin/bash
# A/B of library builds (SF_LIB) on the GPU box: interleaved bench lines (timing) and, with PMC=1, one
# rocprofv3 --pmc pass per build of the LDS / issue counters of the trace kernel.
# Usage (on the box, repo root): [REPS=3] [PMC=1] scripts/lib_ab.sh <tag> "<bench args>" <lib.so>[@flags] ...
#   REPS=0: no timing runs; lib.so@0x100 runs that library with SF_FLAGS=0x100
set -e
TAG=${1:-libab}; shift; ARGS=$1; shift
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-3}); do
  for LF in "$@"; do
    L=${LF%@*}; F=0; [ "$L" != "$LF" ] && F=${LF#*@}
    SF_LIB_PARTIAL=1 SF_FLAGS=$F SF_LIB=$R/$L timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --steps 200 --warmup 30 $ARGS > $OUT/b.json
    python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$LF', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'clk', j['roofline'].get('clock_mhz_live'), 'Mrays', j['value'], 'fixed', j['fixed_camera']['frame_ms'] if j.get('fixed_camera') else None)"
  done
done
if [ "${PMC:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  i=0
  for LF in "$@"; do
    L=${LF%@*}; F=0; [ "$L" != "$LF" ] && F=${LF#*@}
    i=$((i+1))
    SF_LIB_PARTIAL=1 SF_FLAGS=$F SF_LIB=$R/$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc$i -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras $ARGS > $OUT/pmc$i.log 2>&1
    echo "== $LF"
    python3 $R/scripts/pmc_summary.py $OUT/pmc$i | grep -A12 "sf_trace_queue[12] " || true
  done
fi
