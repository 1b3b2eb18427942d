#!/bin/bash
# round 6: sf_dist_set_view applied lazily per slot (new lib) vs on every slot per frame (scratch_ab/lib_old.so):
# the dist tests, then the bench's member-share leg A/B, alternating
set -o pipefail
O=gpurun_out/${TAG:-r6lv}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_frames.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2 3; do
  for lib in old new; do
    if [ $lib = old ]; then export SF_LIB=$PWD/scratch_ab/lib_old.so; else unset SF_LIB; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b_$lib.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$O/b_$lib.json').read().strip().splitlines()[-1]); m=d['member_shares']; print('$lib', d['ms_per_step'], ' '.join(f\"{k}: {m[k]['steady_ms']} ({m[k]['speedup']}x)\" for k in ('n2','n4','n8')))" | tee -a $O/ab.txt
  done
done
