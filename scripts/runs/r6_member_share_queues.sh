#!/bin/bash
# round 6: which hardware queues the 1/8 share's slot streams land on, fresh vs after a 4-slot dist was made and closed
# (kernel trace: Queue_Id / Stream_Id per dispatch), plus untraced timings of PRE=n2 / n8 / a torch stream
set -o pipefail
R=$PWD; O=$R/gpurun_out/${TAG:-r6msqq}; mkdir -p $O
for pre in "n2" "n8"; do
  echo "PRE=$pre" | tee -a $O/untraced.txt
  PRE=$pre timeout -k 10 300 python3 -u scripts/member_share_probe.py 8 600 1 2>&1 | grep -v amdgpu.ids | tee -a $O/untraced.txt || exit 1
done
cd /tmp && export TMPDIR=/tmp
for pre in "" "n4"; do
  PRE=$pre timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_${pre:-fresh} -o run --output-format csv -- python3 $R/scripts/member_share_probe.py 8 600 1 > $O/traced_${pre:-fresh}.txt 2>&1 || exit 1
done
