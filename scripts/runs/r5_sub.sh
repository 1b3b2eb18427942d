#!/bin/bash
# Subtree-split tiles: parity (new tests, random views), the GPU suite, share probes and bench lines A/B.
set -e
OUT=gpurun_out/r5sub; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_subtree.py tests/test_gpu_random_views.py -x -q -k "subtree" --timeout 120 --timeout-method thread > $OUT/pytest_sub.log 2>&1 || { tail -40 $OUT/pytest_sub.log; exit 1; }
tail -1 $OUT/pytest_sub.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
export PROBE_SLOTS=4 PROBE_N=1,4,8 PROBE_SPLITS=auto
timeout -k 10 200 python3 -u scripts/share_probe.py > $OUT/share_base.txt 2>&1; grep x $OUT/share_base.txt
SF_ORDER=1 SF_SPLIT_PARTS=4 timeout -k 10 200 python3 -u scripts/share_probe.py > $OUT/share_q.txt 2>&1; grep x $OUT/share_q.txt
SF_ORDER=1 SF_SPLIT_PARTS=subtree timeout -k 10 200 python3 -u scripts/share_probe.py > $OUT/share_sub.txt 2>&1; grep x $OUT/share_sub.txt
PROBE_SPLITS=model SF_ORDER=1 SF_SPLIT_PARTS=subtree timeout -k 10 200 python3 -u scripts/share_probe.py > $OUT/share_submodel.txt 2>&1; grep x $OUT/share_submodel.txt
for v in base sub; do
  if [ $v = sub ]; then export SF_SPLIT_PARTS=subtree SF_SPLIT_BUCKETS=model; fi
  for st in 20 200; do
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps $st --warmup 5 > $OUT/b_${v}_$st.json 2>/dev/null
    python3 -c "import json; j=json.loads(open('$OUT/b_${v}_$st.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('$v', $st, 'frame', j['frame_ms'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', j['frame_latency_ms'], 'exact', j['check']['bit_exact'])"
  done
done
