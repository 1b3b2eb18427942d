#!/bin/bash
# round 6: the 16-queue / 8-slots-for-tiny-shares policy -- share curve at the bench's policy, c1 at 8 vs 4 in flight,
# the default bench line, a 20-step line, and the two-rank rehearsal of the dist flow on one GPU
set -o pipefail
O=gpurun_out/${TAG:-r6qp2}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | tee -a $O/share.txt || exit 1
done
for r in 1 2; do
  for sl in 0 4; do
    timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --width 640 --height 360 --K 1.0 --slots $sl > $O/c1.json 2>/dev/null || exit 1
    python3 -c "import json; j=json.loads(open('$O/c1.json').read().strip().split(chr(10))[-1]); p=j['pipeline']; print('c1 slots $sl', j['config'].get('slots'), j['config'].get('hw_queues'), 'frame', j['frame_ms'], 'steady', p['steady_frame_ms'], 'lat', j['frame_latency_ms'], 'exact', j['check']['bit_exact'])" | tee -a $O/c1.txt
  done
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_$i.json 2> $O/bench20.err || exit 1
done
for f in bench1 bench20_1 bench2 bench20_2; do python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); p=d['pipeline']; print('$f', d['value'], d['ms_per_step'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', d['frame_latency_ms'], 'exact', d['check']['bit_exact'], 'slots', d['config'].get('slots'), d['config'].get('hw_queues'))"; done
timeout -k 10 400 python -u bench.py --gpus 2 --rehearse --steps 20 --warmup 5 --no-cpu-baseline > $O/rehearse2.json 2> $O/rehearse2.err || { tail -20 $O/rehearse2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/rehearse2.json').read().strip().splitlines()[-1]); print('rehearse2', d['value'], d['ms_per_step'], d['config'].get('parallelism'), d['check']['bit_exact'])"
