#!/bin/bash
# round 6: context streams on queues of their own (CU-masked, SF_STREAM_CUMASK=1, the default) vs plain streams on the
# runtime's shared queues (0): the bench's 20-step line and member shares interleaved, the default line each, the
# GPU suite with the default
set -o pipefail
O=gpurun_out/${TAG:-r6cm}; mkdir -p $O
line() {  # line <label> <file>
  python3 -c "import json; d=json.loads(open('$2').read().strip().splitlines()[-1]); m=d['member_shares']; p=d['pipeline']; print('$1', d['value'], d['ms_per_step'], 'steady', p['steady_frame_ms'], 'lat', d['frame_latency_ms'], 'exact', d['check']['bit_exact'], ' '.join(f\"{k}: {m[k]['steady_ms']} ({m[k]['speedup']}x)\" for k in ('n2','n4','n8')))" | tee -a $O/cumask.txt
}
for r in 1 2; do
  for cm in 1 0; do
    SF_STREAM_CUMASK=$cm timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b20_$cm.json 2> $O/b20_$cm.err || exit 1
    line "cumask=$cm 20-step" $O/b20_$cm.json
  done
done
for cm in 1 0; do
  SF_STREAM_CUMASK=$cm timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/b200_$cm.json 2> $O/b200_$cm.err || exit 1
  line "cumask=$cm 200-step" $O/b200_$cm.json
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
