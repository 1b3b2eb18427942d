#!/bin/bash
# Submit one command to the GPU box via gpurun. Resubmits only when gpurun reports the call as
# "transient" (box not obtained: not charged, nothing ran); never re-runs a command that ran.
# Usage: scripts/gpu.sh <timeout_s> '<command>'   (GPU_TRIES attempts, default 12, GPU_WAIT s apart, default 120)
T=$1; shift
TRIES=${GPU_TRIES:-12}; WAIT=${GPU_WAIT:-120}
for i in $(seq $TRIES); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_last.txt 2>&1
  st=$(python3 -c "import json; print(json.load(open('/root/repo/gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  tail -2 /tmp/gpurun_last.txt
  if [ "$st" != "transient" ]; then echo "status=$st"; exit 0; fi
  echo "transient (attempt $i), waiting"; sleep $WAIT
done
