#!/bin/bash
# round 6: the batch-8 policy for tiny band shares -- the multi-frame tests, the bench's default line with the projected
# member shares, a 20-step line, the two-rank rehearsal
set -o pipefail
O=gpurun_out/${TAG:-r6bp}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_frames.txt 2>&1 || { tail -30 $O/pytest_frames.txt; exit 1; }
tail -1 $O/pytest_frames.txt
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1]); m=d['member_shares']; print('bench', d['value'], d['ms_per_step'], 'steady', d['pipeline']['steady_frame_ms'], ' '.join(f\"{k}: {m[k]['steady_ms']} ({m[k]['speedup']}x, {m[k]['slots']} slots, batch {m[k]['frames_per_launch']}, 64 steps {m[k]['ms_per_step']})\" for k in ('n2','n4','n8')))" | tee -a $O/policy.txt
done
timeout -k 10 400 python -u bench.py --gpus 2 --rehearse --steps 20 --warmup 5 --no-cpu-baseline > $O/rehearse2.json 2> $O/rehearse2.err || { tail -20 $O/rehearse2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/rehearse2.json').read().strip().splitlines()[-1]); print('rehearse2', d['value'], d['ms_per_step'], d['config']['slots'], d['config']['frames_per_launch'], d['check']['bit_exact'])" | tee -a $O/policy.txt
