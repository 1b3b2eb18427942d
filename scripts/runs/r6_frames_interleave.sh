#!/bin/bash
# round 6: multi-frame launches with the whole sequence frame-interleaved (SF_FRAMES_HEAVY >= units: position G is
# frame G % n, order position G / n). Tickets of queue k are = k mod 32 and the grid is a multiple of n, so a wave
# only ever sees frame blockIdx % n: no frame switches. 16 hardware queues.
set -o pipefail
O=gpurun_out/${TAG:-r6fi}; mkdir -p $O
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
  echo "== heads (default)" | tee -a $O/frames_interleave.txt
  timeout -k 10 300 python3 -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --reps 3 --configs 8:1,16:8,16:4 2>&1 | grep -v amdgpu.ids | tee -a $O/frames_interleave.txt || exit 1
  echo "== interleaved" | tee -a $O/frames_interleave.txt
  SF_FRAMES_HEAVY=100000000 timeout -k 10 300 python3 -u scripts/frames_probe.py 1920 1080 0.25 --share 8 --reps 3 --configs 8:1,16:8,16:4 2>&1 | grep -v amdgpu.ids | tee -a $O/frames_interleave.txt || exit 1
done
echo "== interleaved, 1/4 shares and whole frames" | tee -a $O/frames_interleave.txt
SF_FRAMES_HEAVY=100000000 timeout -k 10 300 python3 -u scripts/frames_probe.py 1920 1080 0.25 --share 4 --reps 3 --configs 4:1,16:8,8:4 2>&1 | grep -v amdgpu.ids | tee -a $O/frames_interleave.txt || exit 1
SF_FRAMES_HEAVY=100000000 timeout -k 10 300 python3 -u scripts/frames_probe.py 1920 1080 0.25 --reps 3 --configs 3:1,8:4,16:8 2>&1 | grep -v amdgpu.ids | tee -a $O/frames_interleave.txt || exit 1
