#!/bin/bash
# round 6: the process-wide context stream pool (SF_STREAM_POOL, default on) against a stream per context: the 1/8
# share after the bench's earlier legs, the bench's member-share leg, and the GPU suite with the pool
set -o pipefail
O=gpurun_out/${TAG:-r6pool}; mkdir -p $O
for r in 1 2; do
  for pool in 1 0; do
    for pre in "n2,n4" "main,c4,n2,n4"; do
      echo -n "pool=$pool PRE=$pre: " | tee -a $O/pool.txt
      SF_STREAM_POOL=$pool PRE=$pre timeout -k 10 200 python3 -u scripts/member_share_probe.py 8 600 1 2>&1 | grep "N=8 slots" | cut -c1-64 | tee -a $O/pool.txt || exit 1
    done
  done
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); m=d['member_shares']; print('bench', d['ms_per_step'], ' '.join(f\"{k}: {m[k]['steady_ms']} ({m[k]['speedup']}x)\" for k in ('n2','n4','n8')))" | tee -a $O/pool.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
