#!/bin/bash
# Quick iteration probe: core parity subset, bench lines (c3 moving + c1), one PMC pass on the trace kernel.
# Usage (on the box, repo root): scripts/perf_probe.sh <tag> [ENV=..]
set -e
TAG=${1:-pp}; shift || true
R=$PWD; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_views.py -x -q -k "tiny or config_frames or random or progressive_matches or split" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in "" "--width 640 --height 360 --K 1.0"; do
  env "$@" timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --steps 200 --warmup 30 $cfg > $OUT/b.json
  python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('${cfg:-c3}', 'frame', j['frame_ms'], 'trace', j['roofline']['kernel_ms'], 'Mrays', j['value'], 'fixed', j['fixed_camera']['frame_ms'] if j.get('fixed_camera') else None)"
done
cd /tmp && export TMPDIR=/tmp
env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SMEM -d $OUT/pmc -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > $OUT/pmc.log 2>&1
python3 $R/scripts/pmc_summary.py $OUT/pmc | grep -A10 "sf_trace_queue[12] "
