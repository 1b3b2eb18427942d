#!/bin/bash
# round 6: is the 1/8 share slowed by the number of hardware queues that exist in the process (idle ones included)?
# extra idle queues before a fresh 8-slot dist, and the bench's legs before it at GPU_MAX_HW_QUEUES 8 / 12 / 16
set -o pipefail
O=gpurun_out/${TAG:-r6hwq}; mkdir -p $O
run() {  # run <label> <env...>
  local label=$1; shift
  echo "$label" | tee -a $O/hwq.txt
  env "$@" timeout -k 10 300 python3 -u scripts/member_share_probe.py 8 600 1 2>&1 | grep -v amdgpu.ids | tee -a $O/hwq.txt || exit 1
}
run "fresh, 16 queues" GPU_MAX_HW_QUEUES=16
run "1 extra stream, 16 queues" GPU_MAX_HW_QUEUES=16 EXTRA_STREAMS=1
run "4 extra streams, 16 queues" GPU_MAX_HW_QUEUES=16 EXTRA_STREAMS=4
run "PRE bench legs, 8 queues" GPU_MAX_HW_QUEUES=8 SF_HW_QUEUES=8 PRE=main,c4,n2,n4
run "fresh, 8 queues" GPU_MAX_HW_QUEUES=8
run "PRE n2,n4, 12 queues" GPU_MAX_HW_QUEUES=12 SF_HW_QUEUES=12 PRE=n2,n4
run "PRE n2,n4, 8 queues" GPU_MAX_HW_QUEUES=8 SF_HW_QUEUES=8 PRE=n2,n4
