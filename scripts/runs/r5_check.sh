#!/bin/bash
# Round-5 GPU pass: parity suite, smoke, one bench line. Every GPU step under its own limit; stop at the first failure.
# Usage (on the box): scripts/r5_check.sh <tag> [bench args...]
set -e
TAG=${1:-r5}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > $OUT/bench20.json 2> $OUT/bench20.err
python3 -c "import json,sys; d=json.loads(open('$OUT/bench20.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['frame_latency_ms'], d['pipeline'], d['check']['bit_exact'], d['roofline']['clock_mhz_live'])"
